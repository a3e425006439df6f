#!/bin/bash
# Knock-outs of conv_halo3_kernel (diagnostic): library copies built with
# -DEEGAN_HALO_KNOCK=bits (1 no loads, 2 no stores, 4 no MFMAs) into
# tools/ab_lib/ (build on the CPU side first: tools/gpu_halo_knock.sh build),
# conv_bench of the 3x3 shapes with each.
S=${S:-c3x3_64_128,c3x3_128_64,c3x3_256_32,d256_b0_3x3,d256_b1_3x3,d256_b2_3x3}
if [ "$1" = build ]; then
  cd ee-gan_amd/csrc && mkdir -p ../../tools/ab_lib
  for k in ${KNOCKS:-1 2 3 4 6}; do
    /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -DEEGAN_HALO_KNOCK=$k -c conv.hip -o build/conv_k$k.o &&
    /opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o ../../tools/ab_lib/libeegan_hip_knock$k.so build/conv_k$k.o \
      $(ls build/*.o | grep -v '/conv') || exit 1
  done
  exit 0
fi
source ./run_gpu_steps.sh
TAG=${1:-hk}
step 200 ${TAG}_k0 python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
for k in ${KNOCKS:-1 2 3 4 6}; do
  step 200 ${TAG}_k$k env EEGAN_HIP_LIB=$PWD/tools/ab_lib/libeegan_hip_knock$k.so python3 tools/conv_bench.py --shapes $S --dirs fwd,bwdd --device-time
done
for k in 0 ${KNOCKS:-1 2 3 4 6}; do echo "== knock $k"; grep -h 'TF/s' gpurun_out/${TAG}_k$k.log; done
# D256's d_update alone, kernel by kernel (rocprofv3 kernel trace, one stream)
if [ -n "$LANE" ]; then
  cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
  step 300 ${TAG}_lt_d2 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_lt_d2 -o run -- python3 tools/lane_trace.py --d 2
  LANE_TOP=40 python3 tools/lane_trace.py --report gpurun_out/${TAG}_lt_d2 > gpurun_out/${TAG}_lt_d2_report.txt
  find gpurun_out/${TAG}_lt_d2 -name '*.csv' -delete
  step 300 ${TAG}_lt_all rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_lt_all -o run -- python3 tools/lane_trace.py --d -1
  LANE_TOP=40 python3 tools/lane_trace.py --report gpurun_out/${TAG}_lt_all > gpurun_out/${TAG}_lt_all_report.txt
  find gpurun_out/${TAG}_lt_all -name '*.csv' -delete
fi
