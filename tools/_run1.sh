set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
APM_DF_SPLIT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "dataflow or mixed or fp16x3" > gpurun_out/t_df.txt 2>&1 || { tail -30 gpurun_out/t_df.txt; exit 1; }
tail -1 gpurun_out/t_df.txt
bash tools/phases.sh APM_DF_SPLIT 1 0 > gpurun_out/ph.txt 2>&1
grep -E "^==|^hash|theta-call wall|newton \(|panel_df" gpurun_out/ph.txt
APM_LIB=$PWD/tools/_wpe2/libapm.so bash tools/phases.sh APM_DF_SPLIT 1 > gpurun_out/ph2.txt 2>&1
echo "wpe2:"; grep -E "^==|^hash|theta-call wall|newton \(|panel_df" gpurun_out/ph2.txt
