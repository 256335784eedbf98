# Build the working tree's render kernel (or $2, a .hip file) as raytracinginaweekend_amd/librtw_$1.so for
# A/B runs (extra compiler flags from $RTW_VARIANT_FLAGS)
set -e
cd "$(dirname "$0")/../raytracinginaweekend_amd/csrc"
src=${2:-rtw_device.hip}
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize $RTW_VARIANT_FLAGS -c -x hip $src -o build/ab_$1.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../librtw_$1.so build/ab_$1.o build/scene_builder.o \
  build/demo_worlds.o build/rtw_common.o build/rtw_sort.o build/rtw_sah.o build/rtw_multi.o
rm -f build/ab_$1.o
