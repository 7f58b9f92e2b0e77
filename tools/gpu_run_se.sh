set -e
mkdir -p gpurun_out/se1
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/se1/pytest.log 2>&1 || { tail -40 gpurun_out/se1/pytest.log; exit 1; }
tail -2 gpurun_out/se1/pytest.log
bash tools/variant_ab.sh se1 bash tools/single_probe.sh gpurun_out/sp_se1
for v in se0 se1; do head -2 gpurun_out/var_se1/$v.txt; done
