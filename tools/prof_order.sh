set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/prof_order
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_order -o run -- python3 tools/ab.py --config 3 --rounds 1 --frames 20 --variants default > gpurun_out/prof_order/ab.txt 2>&1
