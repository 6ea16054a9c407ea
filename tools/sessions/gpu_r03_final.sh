set -o pipefail
mkdir -p gpurun_out/fE
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/fE/smoke.txt 2>&1 || { tail -20 gpurun_out/fE/smoke.txt; exit 1; }
tail -1 gpurun_out/fE/smoke.txt
bash tools/gpu_r03.sh fE tests bench:config2 bench:aead bench:encap bench:decap_host
