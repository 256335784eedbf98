# Register / scratch report of the product render kernels (compile-only, no GPU):
#   bash tools/resources.sh > profiles/r06/resources.txt
cd "$(dirname "$0")/../raytracinginaweekend_amd/csrc"
/opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 -ffp-contract=off -fno-fast-math --offload-arch=gfx950 \
  -fhip-fp32-correctly-rounded-divide-sqrt -munsafe-fp-atomics -fno-slp-vectorize -c -x hip rtw_device.hip \
  -o /tmp/rtw_res.o -Rpass-analysis=kernel-resource-usage 2>&1 \
  | grep -E "remark: .*(Function Name|VGPRs:|ScratchSize|VGPRs Spill|SGPRs Spill|Occupancy|LDS Size)" \
  | sed 's/.*remark: //; s/ \[-Rpass.*//' | paste - - - - - - - | grep "render_kernel" \
  | sed 's/Function Name: _ZN12_GLOBAL__N_113render_kernelILb\([01]\)ELi\([0-9]\)ELi\([0-9]\)ELi\([0-9]\)ELb\([01]\)ELb\([01]\)EEEvNS_5KArgsE/render_kernel<STATS=\1, LDS=\2, LK=\3, TX=\4, GEN=\5, WP=\6>/'
