# Round-5 development check on one MI355X: selected GPU tests (stop on a crash), an optional
# short bench, and the stationary 64-chain theta-call timeline of tools/time_theta.py.
#   bash tools/r05_check.sh "<pytest -k expression | all | none>" "<bench args | none>"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O
K="$1"
if [ "$K" = "all" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
  rc=$?
elif [ "$K" != "none" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $O/tests.txt 2>&1
  rc=$?
else
  rc=0
fi
[ "$K" != "none" ] && tail -3 $O/tests.txt && grep -E "FAILED|Error" $O/tests.txt | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stop"; exit $rc; fi
if [ "$2" != "none" ]; then
  timeout -k 10 600 python -u bench.py $2 > $O/bench.json 2> $O/bench.err
  rc=$?; echo "bench exit $rc"; tail -3 $O/bench.err
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
fi
timeout -k 10 300 python -u tools/time_theta.py --batch 64 --reps 3 --theta-file profiles/r04_stationary_thetas.npy > $O/stat_theta.txt 2>&1 || exit $?
head -4 $O/stat_theta.txt
echo done
