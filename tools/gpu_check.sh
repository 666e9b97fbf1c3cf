set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
rocm-smi --showproductname > gpurun_out/smi.txt 2>&1 || true
nproc > gpurun_out/nproc.txt; lscpu | head -20 >> gpurun_out/nproc.txt
timeout -k 10 240 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo SMOKE_FAIL; cat gpurun_out/smoke.log | tail -30; exit 1; }
timeout -k 10 600 python -m pytest tests -m gpu -q -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --cpu-seconds 8 > gpurun_out/bench.json 2> gpurun_out/bench.err; rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
