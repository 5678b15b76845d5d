# hipBLASLt trailing-update path (APM_GEMM) on one MI355X: standalone update timings of both
# paths, then the stationary 64-chain theta-call A/B in one process, then the precision tests
# with the GEMM path on.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
bash tools/r05_upd.sh || exit $?
timeout -k 10 300 python -u tools/ab_knob.py APM_GEMM 0 1 0 1 --reps 3 > $O/ab_gemm.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/ab_gemm.txt; [ $rc -ne 0 ] && exit $rc
APM_GEMM=1 timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "mixed or config2 or config4 or fp16x3 or dataflow or forced" > $O/gemm_tests.txt 2>&1
rc=$?; tail -3 $O/gemm_tests.txt; grep FAILED $O/gemm_tests.txt
exit $rc
