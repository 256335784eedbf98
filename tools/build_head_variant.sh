# Build the committed (HEAD or $2) render kernel as raytracinginaweekend_amd/librtw_$1.so for A/B runs
# (extra compiler flags, e.g. -DRTW_QUEUES=32, from $RTW_VARIANT_FLAGS)
set -e
cd "$(dirname "$0")/../raytracinginaweekend_amd/csrc"
git show ${2:-HEAD}:raytracinginaweekend_amd/csrc/rtw_device.hip > ab_tmp.hip
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize $RTW_VARIANT_FLAGS -c -x hip ab_tmp.hip -o build/ab_tmp.o
rm -f ab_tmp.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../librtw_$1.so build/ab_tmp.o build/scene_builder.o \
  build/demo_worlds.o build/rtw_common.o build/rtw_sort.o build/rtw_sah.o build/rtw_multi.o
