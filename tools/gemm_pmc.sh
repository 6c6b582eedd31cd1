# PMC passes on GEMM kernels (tools/gemm_one_modes.py <modes>), one counter group per pass, each
# under its own time limit; summary -> gpurun_out/<tag>/summary.json
set -o pipefail
TAG=${1:-gemm_pmc}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
i=0
for CNT in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-include-regex gemm -d $OUT/p$i -o p --output-format csv -- python tools/gemm_one_modes.py "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python tools/pmc_kernels.py $(find $OUT/p1 -name "*counter_collection.csv") $(find $OUT/p2 -name "*counter_collection.csv") > $OUT/summary.json
python - $OUT/summary.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for k, v in d.items():
    print(k[:60], {x: v.get(x) for x in ("mfma_busy_frac", "sq_wait_inst_any_frac", "sq_wait_inst_lds_frac", "lds_conflict_frac", "SQ_INSTS_LDS", "SQ_INSTS_MFMA", "SQ_INSTS_VALU", "dispatches")})
PY
