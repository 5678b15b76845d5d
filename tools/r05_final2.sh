# Round-5 record in one call: GPU suite + smoke, the round profile (kernel trace + PMC passes of the
# default bench), its PMC summary installed as profiles/r05_pmc_traffic.json on the box so that the
# bench that follows (the driver's invocation) finds a current pmc_provenance, the Newton-only PMC
# passes and a stationary theta-call timeline
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05fin; mkdir -p $O
bash tools/r05_gputests.sh > $O/tests.out 2>&1 || { echo "tests failed"; tail -20 $O/tests.out; exit 1; }
tail -3 $O/tests.out
bash tools/profile_round.sh > $O/profile_round.log 2>&1 || { echo "profile_round failed"; tail -20 $O/profile_round.log; exit 1; }
cp gpurun_out/prof_round/window.json profiles/r05_pmc_traffic.json
echo "profile done"
timeout -k 10 900 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || { echo "bench failed"; tail -20 $O/bench20.err; exit 1; }
echo "bench done"; tail -c 300 $O/bench20.json
bash tools/r05_pmc_newton.sh > $O/pmc_newton.log 2>&1 || { echo "pmc newton failed"; tail -5 $O/pmc_newton.log; exit 1; }
echo "pmc done"
bash tools/r05_timeline.sh > $O/timeline.log 2>&1 || { echo "timeline failed"; exit 1; }
echo "timeline done"
