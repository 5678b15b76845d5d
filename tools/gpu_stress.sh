# configs[4] stress (N=16384 D=64 N_imp=1024, 8 chains) + a full-size oracle check at N=8192
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chains.py -x -v --timeout 240 --timeout-method thread > gpurun_out/chains.log 2>&1 && \
timeout -k 10 400 python -u tools/stress.py --batch 8 --reps 2 > gpurun_out/stress16k.json 2> gpurun_out/stress16k.err && \
timeout -k 10 400 python -u tools/stress.py --n 8192 --batch 1 --reps 2 --check 1 > gpurun_out/stress8k_check.json 2> gpurun_out/stress8k_check.err
