# PMC passes (one counter group per rocprofv3 run) for both scenes at 1080p x SPP
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for SC in final_scene1 suzanne; do
D=gpurun_out/pmc_$SC; mkdir -p $D
P="python3 tools/prof_render.py --scene $SC --spp ${SPP:-32}"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $D/kt -o kt --output-format csv -- $P > $D/kt.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES -d $D/p1 -o p1 --output-format csv -- $P > $D/p1.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d $D/p2 -o p2 --output-format csv -- $P > $D/p2.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_ADDR_CONFLICT SQ_INST_LEVEL_VMEM SQ_CYCLES -d $D/p5 -o p5 --output-format csv -- $P > $D/p5.log 2>&1 || exit $?
python3 tools/pmc_summary.py $D > $D/summary.txt 2>&1
done
