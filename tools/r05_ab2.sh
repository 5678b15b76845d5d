# Round-5 A/B batch 2: one-panel lookahead of the Newton factorisation (APM_LOOKAHEAD) on the
# stationary 64-chain theta-call (bitwise equal outputs expected), the Newton/precision tests with
# it on, then the Newton-only PMC passes (tools/r05_pmc_newton.sh).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
timeout -k 10 300 python -u tools/ab_knob.py APM_LOOKAHEAD 0 1 0 1 --reps 3 > $O/ab_la.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/ab_la.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "mixed or config2 or fp16x3 or dataflow or forced or batch" > $O/la_tests.txt 2>&1
rc=$?; tail -2 $O/la_tests.txt; grep FAILED $O/la_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r05_pmc_newton.sh
