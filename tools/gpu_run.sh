#!/bin/bash
# One GPU call built from steps, run in order on the box; the first step that ends
# on a signal, a time limit or a crash ends the call (no retries, no further GPU step).
#
#   bash tools/gpu_run.sh TAG STEP [STEP ...]      (inside gpurun, from the repo root)
#
# STEP forms (outputs under gpurun_out/, named by TAG):
#   smoke                          __graft_entry__.smoke()
#   pytest:SELECTION               python -m pytest SELECTION -m gpu (-> TAG_pytest.log; -k "$PYTEST_K" if set)
#   bench:NAME:ARGS                python bench.py ARGS            (-> TAG_NAME.json / .err)
#   prof:NAME:ARGS                 rocprofv3 --kernel-trace --stats of bench.py ARGS (-> TAG_NAME_prof/)
#   py:NAME:ARGS                   python ARGS                      (-> TAG_NAME.out / .err)
# A step's limit is STEP_TIMEOUT seconds (default 300). A pytest failure (exit 1)
# does not stop the call; bench / py exits other than 0 do.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1
shift
LIM=${STEP_TIMEOUT:-300}
fatal() {  # exit codes that mean the GPU or the process died: stop here
    case $1 in 124|134|137|139|143) return 0 ;; esac
    [ "$1" -gt 128 ] && return 0
    return 1
}
for step in "$@"; do
    kind=${step%%:*}
    rest=${step#*:}
    name=${rest%%:*}
    args=${rest#*:}
    case $kind in
        smoke)
            timeout -k 10 "$LIM" python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/${TAG}_smoke.log" 2>&1
            rc=$?; echo "smoke rc=$rc"; tail -2 "gpurun_out/${TAG}_smoke.log"
            [ $rc -eq 0 ] || exit $rc ;;
        pytest)
            timeout -k 10 "$((LIM * 4))" python -u -m pytest $rest ${PYTEST_K:+-k "$PYTEST_K"} -m gpu -v -rf \
                --timeout 240 --timeout-method thread \
                > "gpurun_out/${TAG}_pytest.log" 2>&1
            rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|ERROR" "gpurun_out/${TAG}_pytest.log" | tail -25
            if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi ;;
        bench)
            timeout -k 10 "$LIM" python bench.py $args > "gpurun_out/${TAG}_${name}.json" 2> "gpurun_out/${TAG}_${name}.err"
            rc=$?; echo "bench $name rc=$rc"; cut -c1-600 "gpurun_out/${TAG}_${name}.json"
            [ $rc -eq 0 ] || { tail -5 "gpurun_out/${TAG}_${name}.err"; exit $rc; } ;;
        prof)
            timeout -s KILL "$LIM" rocprofv3 --kernel-trace --stats --output-format csv -d "gpurun_out/${TAG}_${name}_prof" -o run \
                -- python bench.py $args > "gpurun_out/${TAG}_${name}_prof.log" 2>&1
            rc=$?; echo "prof $name rc=$rc"
            fatal $rc && exit $rc ;;
        py)
            timeout -k 10 "$LIM" python $args > "gpurun_out/${TAG}_${name}.out" 2> "gpurun_out/${TAG}_${name}.err"
            rc=$?; echo "py $name rc=$rc"; tail -c 1500 "gpurun_out/${TAG}_${name}.out"
            [ $rc -eq 0 ] || { tail -5 "gpurun_out/${TAG}_${name}.err"; exit $rc; } ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done
