cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-timer > gpurun_out/gaps.log 2>&1
python3 tools/trace_gaps.py gpurun_out/gaps
find gpurun_out/gaps -name '*.csv' -size +20M -delete
