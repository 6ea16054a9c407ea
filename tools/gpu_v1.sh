set -o pipefail
T=${1:-v2}
mkdir -p gpurun_out/$T
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_encap.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/$T/pytest.txt 2>&1 || { tail -30 gpurun_out/$T/pytest.txt; exit 1; }
tail -2 gpurun_out/$T/pytest.txt
timeout -k 10 500 python3 -u tools/ab.py encap encap_parts=1 encap_parts=2,encap_occ=3 encap_parts=4,encap_occ=3 encap_parts=8,encap_occ=3 encap_parts=4,encap_occ=2 encap_parts=4 > gpurun_out/$T/ab_encap.json 2>&1 || { tail -30 gpurun_out/$T/ab_encap.json; exit 1; }
tail -1 gpurun_out/$T/ab_encap.json
