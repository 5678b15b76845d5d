# the InvalidCovarianceMatrixError tests and the configs[2] / stationary parity tests
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05icm; mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_errors.py tests/test_gpu_configs.py -k "invalid_cov or reference_route or config2 or errors" 2>&1 | tee $O/tests.txt
