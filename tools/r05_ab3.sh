# Round-5 check 3: swizzled fp16x3 LDS layout - standalone update timings and hashes (must equal
# profiles/r05_update_vs_hipblaslt.txt's), the stationary theta-call (hash e3a88ef092ca expected),
# the Newton tests, then the Newton-only PMC passes again.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
bash tools/r05_upd.sh "" _swz || exit $?
timeout -k 10 300 python -u tools/ab_knob.py APM_LOOKAHEAD 1 0 1 --reps 3 > $O/ab_swz.txt 2>&1; rc=$?
grep -v amdgpu.ids $O/ab_swz.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "mixed or config2 or fp16x3 or dataflow or forced or batch" > $O/swz_tests.txt 2>&1
rc=$?; tail -2 $O/swz_tests.txt; grep FAILED $O/swz_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash tools/r05_pmc_newton.sh
