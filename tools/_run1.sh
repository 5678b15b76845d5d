set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
APM_LIB=$PWD/tools/_oldlib/libapm_dftrace.so timeout -k 10 200 python -u tools/df_trace.py > gpurun_out/df_trace.txt 2>&1
cat gpurun_out/df_trace.txt
