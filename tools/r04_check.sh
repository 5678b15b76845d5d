# Round-4 development check on one MI355X: GPU tests (stop on a crash, go on after plain test
# failures), then phase timelines of one 64-chain theta-call under knob settings.
#   bash tools/r04_check.sh "<pytest -k expression or empty>" "VAR=v1,v2 VAR2=v3,v4"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
K="$1"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/r04_tests.txt 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/r04_tests.txt 2>&1
fi
rc=$?
tail -3 gpurun_out/r04_tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stop"; exit $rc; fi
for spec in $2; do
  VAR=${spec%%=*}; VALS=${spec#*=}
  bash tools/phases.sh $VAR ${VALS//,/ } || exit $?
done
