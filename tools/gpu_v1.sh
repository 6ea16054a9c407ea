set -o pipefail
T=${1:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -30 gpurun_out/$T/pytest.txt; exit 1; }
tail -1 gpurun_out/$T/pytest.txt
timeout -k 10 500 python3 -u tools/ab.py aead aead_pair=1 aead_pair=2 aead_pair=3 > gpurun_out/$T/ab_aead.json 2>&1 || { tail -30 gpurun_out/$T/ab_aead.json; exit 1; }
tail -1 gpurun_out/$T/ab_aead.json
timeout -k 10 500 python3 -u tools/ab.py encap aead_pair=1 aead_pair=3 > gpurun_out/$T/ab_encap.json 2>&1 || { tail -30 gpurun_out/$T/ab_encap.json; exit 1; }
tail -1 gpurun_out/$T/ab_encap.json
