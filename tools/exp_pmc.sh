#!/bin/bash
R="$GRAFT_REPO_ROOT"
O="$R/gpurun_out/pmc"
mkdir -p "$O"
timeout -k 10 200 python "$R/tools/dump_atrous_inputs.py" /tmp/atrous_in > "$O/dump.log" 2>&1 || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 --list-avail > "$O/avail.txt" 2>&1
for v in 0 6 3; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_ANY --output-format csv -d "$O/v$v" -o run -- "$R/tools/exp_atrous_real" /tmp/atrous_in $v 4 > "$O/v$v.log" 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc SQ_LEVEL_WAVES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d "$O/w$v" -o run -- "$R/tools/exp_atrous_real" /tmp/atrous_in $v 4 > "$O/w$v.log" 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc TA_BUSY_avr TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum --output-format csv -d "$O/t$v" -o run -- "$R/tools/exp_atrous_real" /tmp/atrous_in $v 4 > "$O/t$v.log" 2>&1 || echo "ta pass rc=$?"
done
echo done
