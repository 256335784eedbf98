set -o pipefail
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 -L > gpurun_out/pmc/counters_list.txt 2>&1 || true
P="python tools/prof_render.py --scene ${SCENE:-final_scene1} --spp ${SPP:-32}"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pmc/kt -o kt --output-format csv -- $P > gpurun_out/pmc/kt.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM SQ_WAVE_CYCLES -d gpurun_out/pmc/p1 -o p1 --output-format csv -- $P > gpurun_out/pmc/p1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_BRANCH -d gpurun_out/pmc/p2 -o p2 --output-format csv -- $P > gpurun_out/pmc/p2.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_CYCLES -d gpurun_out/pmc/p5 -o p5 --output-format csv -- $P > gpurun_out/pmc/p5.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc/p3 -o p3 --output-format csv -- $P > gpurun_out/pmc/p3.log 2>&1 && \
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc/p4 -o p4 --output-format csv -- $P > gpurun_out/pmc/p4.log 2>&1
echo rc=$?
