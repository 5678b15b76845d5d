# Round-4 record of HEAD on one MI355X: the whole GPU suite, smoke(), the bench under the
# driver's invocation, then a stationary-regime phase timeline (tools/time_theta.py on the
# long-chain record's chain states). Stops at the first crash / time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/final_tests.txt 2>&1
rc=$?; tail -2 gpurun_out/final_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stop"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.txt 2>&1 || exit $?
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench20.json 2> gpurun_out/final_bench20.err || exit $?
TT_ARGS="--theta-file profiles/r04_stationary_thetas.npy" timeout -k 10 300 bash tools/phases.sh APM_OVERLAP_K 1 > gpurun_out/ph_stat.txt 2>&1
