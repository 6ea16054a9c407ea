set -o pipefail
T=${1:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_aead.py tests/test_gpu_encap.py tests/test_oracle_aead.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -30 gpurun_out/$T/pytest.txt; exit 1; }
tail -1 gpurun_out/$T/pytest.txt
bash tools/gpu_r03.sh $T abuild:nopre:aead,encap
