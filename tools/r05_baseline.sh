# Round-5 baseline of HEAD on one MI355X: GPU suite, smoke, the bench under the driver's
# invocation, the stationary phase timeline, and the 2-rank-on-one-GPU bench three times with its
# whole JSON line kept (the round-4 intermittent parity failure lost its parity block to a
# truncated assertion message). Stops at the first crash / time limit.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05b
O=gpurun_out/r05b
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
rc=$?; tail -2 $O/tests.txt
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with $rc: stop"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || exit $?
timeout -k 10 420 python -u bench.py --steps 20 --warmup 5 > $O/bench20.json 2> $O/bench20.err || exit $?
for i in 1 2 3; do
  APM_DEVICE=0 MASTER_ADDR=127.0.0.1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node=2 --master-addr 127.0.0.1 --master-port 2957$i bench.py --gpus 2 --steps 4 \
    --warmup 1 --chains 4 --n-data 1024 --n-features 8 --n-imp 32 --cpu-baseline 0 \
    > $O/dist$i.json 2> $O/dist$i.err
  rc=$?; echo "dist run $i: exit $rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop"; exit $rc; fi
done
timeout -k 10 300 python -u tools/time_theta.py --batch 64 --reps 3 --theta-file profiles/r04_stationary_thetas.npy > $O/stat_theta.txt 2>&1 || exit $?
echo done
