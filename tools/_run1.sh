set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_knobs.py -x -v --timeout 500 --timeout-method thread > gpurun_out/t_knobs.txt 2>&1 || { tail -30 gpurun_out/t_knobs.txt; exit 1; }
tail -2 gpurun_out/t_knobs.txt
APM_DF_SPLIT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "dataflow or mixed or fp16x3" > gpurun_out/t_df.txt 2>&1 || { tail -30 gpurun_out/t_df.txt; exit 1; }
tail -1 gpurun_out/t_df.txt
bash tools/phases.sh APM_DF_SPLIT 2 0 2 0 > gpurun_out/ph.txt 2>&1
grep -E "^==|^hash|theta-call wall|newton \(|panel_df|bulk32" gpurun_out/ph.txt
