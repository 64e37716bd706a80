#!/bin/bash
# Experiment builds: rc_kernels.hip with extra defines, linked with the default objects into
# raytracing-programs_amd/lib/libraycast_hip_<name>.so (load with RC_HIP_LIB=...).
#   scripts/build_variant.sh NAME -DFOO=1 ...
set -e
cd "$(dirname "$0")/.."
name=$1; shift
make -s raytracing-programs_amd/lib/libraycast_hip.so
O=raytracing-programs_amd/lib/obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off \
  -fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt -Iinclude \
  -Iraytracing-programs_amd/csrc -w "$@" -c raytracing-programs_amd/csrc/rc_kernels.hip -o $O/var_$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC $O/var_$name.o $O/rc_api.o $O/rc_shard.o \
  $O/rc_scene.o -o raytracing-programs_amd/lib/libraycast_hip_$name.so -L/opt/rocm/lib -lrccl \
  -Wl,-rpath,/opt/rocm/lib -lpthread
echo built libraycast_hip_$name.so
