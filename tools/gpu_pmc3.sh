# PMC passes (one counter group per rocprofv3 run) of the render kernel on one scene:
#   SCENE=final_scene1 [W=1920 H=1080] SPP=32 bash tools/gpu_pmc3.sh  -> gpurun_out/pmc3_<scene>/summary.txt
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
SC=${SCENE:-final_scene1}
D=${PMC_OUT:-gpurun_out/pmc3_$SC}; mkdir -p $D
P="python3 tools/prof_render.py --scene $SC --width ${W:-1920} --height ${H:-1080} --spp ${SPP:-32} --repeat 2"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- $P > $D/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES -d $D/p1 -o p1 --output-format csv -- $P > $D/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d $D/p2 -o p2 --output-format csv -- $P > $D/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_VMEM SQ_CYCLES -d $D/p5 -o p5 --output-format csv -- $P > $D/p5.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_FLAT SQ_INSTS_FLAT SQ_IFETCH SQ_IFETCH_LEVEL SQ_LDS_IDX_ACTIVE SQ_INSTS_SENDMSG SQ_WAVE_CYCLES -d $D/p6 -o p6 --output-format csv -- $P > $D/p6.log 2>&1 || true
# memory side (round 5, the verdict's C5 question: what its waiting cycles wait on): vector-memory
# instructions in flight, L1 -> L2 read requests and their latency, L2 hit rate, texture-address busy
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VMEM_RD TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_PENDING_STALL_CYCLES_sum TCC_HIT_sum TCC_MISS_sum -d $D/p7 -o p7 --output-format csv -- $P > $D/p7.log 2>&1 || exit $?
python3 tools/pmc_summary.py $D > $D/summary.txt 2>&1
