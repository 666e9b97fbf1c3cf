set -o pipefail
for b in 0 1; do echo -n "bounces $b: "; timeout -k 10 200 python tools/abf.py --lib2 build_ab/same/librtamd.so --config 3 --inflight 2 --frames 300 --rounds 2 --bounces $b 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1; done
echo -n "persistent: "; timeout -k 10 200 python tools/abf.py --lib2 build_ab/same/librtamd.so --config 3 --inflight 2 --frames 300 --rounds 2 --set2 persistent=1 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
echo -n "persistent b0: "; timeout -k 10 200 python tools/abf.py --lib2 build_ab/same/librtamd.so --config 3 --inflight 2 --frames 300 --rounds 2 --bounces 0 --nocheck --set2 persistent=1 2>&1 | grep -v amdgpu.ids | tail -1 || exit 1
