source ./run_gpu_steps.sh
export EEGAN_PARITY_LOG=$PWD/gpurun_out/r04a_parity_log.txt
step 900 r04a_gputests python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step 400 r04a_bench python3 bench.py --cpu-seconds 5
grep -h '"metric"' gpurun_out/r04a_bench.log | cut -c1-400
