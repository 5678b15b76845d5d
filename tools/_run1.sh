set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 60 ./tools/gram.bin > gpurun_out/gram.txt 2>&1
timeout -k 10 60 ./tools/gram.bin 64 64 >> gpurun_out/gram.txt 2>&1
timeout -k 10 60 ./tools/gram.bin 64 8 >> gpurun_out/gram.txt 2>&1
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "gram or cache_tuple or golden" > gpurun_out/t_gram.txt 2>&1
for L in new w2 old new w2 old; do
  unset APM_LIB APM_UGEMM_W2_MIN
  if [ $L = old ]; then export APM_LIB=$PWD/tools/_oldlib/libapm.so; fi
  if [ $L = w2 ]; then export APM_UGEMM_W2_MIN=1; fi
  timeout -k 10 120 python -u tools/ugemm_bench.py --batches 1,4,8,21,64 --reps 20 2>&1 | sed "s/^/$L /" >> gpurun_out/ugemm_ab.txt
done
