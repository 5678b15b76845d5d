cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/call_latency.py > gpurun_out/lat.log 2>&1 && \
APM_SCHED=spin timeout -k 10 120 python -u tools/call_latency.py >> gpurun_out/lat.log 2>&1 && \
APM_SCHED=yield timeout -k 10 120 python -u tools/call_latency.py >> gpurun_out/lat.log 2>&1 && \
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/bench.json 2> gpurun_out/bench.err && \
APM_SCHED=spin timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --cpu-baseline 0 > gpurun_out/bench_spin.json 2> gpurun_out/bench_spin.err
