#!/bin/bash
# PMC passes (separate rocprofv3 runs, counters only with --kernel-trace) on one frame.
# Usage: tools/run_pmc.sh <tag> [c2|c3]
set -o pipefail
cd /tmp && export TMPDIR=/tmp; cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/$1; mkdir -p $OUT
T="python3 tools/prof_target.py ${2:-c2}"
P() { name=$1; shift; timeout -k 10 ${PASS_TIMEOUT:-240} rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run "$@" -- $T > $OUT/$name.log 2>&1; }
# PASSES="fetch write" (e.g. for the whole C4 frame, ~4 min per pass) runs only those
want() { [ -z "$PASSES" ] || [[ " $PASSES " == *" $1 "* ]]; }
want fetch && { P fetch --pmc FETCH_SIZE || exit 1; }
want write && { P write --pmc WRITE_SIZE || exit 1; }
want valu || { echo done; exit 0; }
P valu --pmc SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES || exit 1
P busy --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU_FLOPS_FP64 SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY || exit 1
if [ -n "$MEMPASS" ]; then  # vector-memory instructions (scratch spills) and L2 behaviour
  P mem --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM TCC_HIT_sum TCC_MISS_sum || exit 1
fi
echo done
