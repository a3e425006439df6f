source ./run_gpu_steps.sh
step 200 bnb_base env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_base.so python3 tools/bn_bench.py
step 200 bnb_new python3 tools/bn_bench.py
step 300 bnb_tests python3 -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q -k "bn or BN or generator or syncbn or step" --timeout 120 --timeout-method thread
grep -h "bwd reduce" gpurun_out/bnb_base.log gpurun_out/bnb_new.log
