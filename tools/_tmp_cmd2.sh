source run_gpu_steps.sh
step 300 kernels python3 -m pytest tests/test_gpu_kernels.py -x -q -k "repack or adam or conv_fwd"
bash tools/_tmp_cmd.sh
