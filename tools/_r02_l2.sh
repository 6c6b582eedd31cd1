set -o pipefail
mkdir -p gpurun_out/r02_l2
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r02_l2/trace -o t --output-format csv -- python tools/gemm_one_shapes.py > gpurun_out/r02_l2/trace.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/r02_l2/hit -o p --output-format csv -- python tools/gemm_one_shapes.py > gpurun_out/r02_l2/hit.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r02_l2/fetch -o p --output-format csv -- python tools/gemm_one_shapes.py > gpurun_out/r02_l2/fetch.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES -d gpurun_out/r02_l2/sq -o p --output-format csv -- python tools/gemm_one_shapes.py > gpurun_out/r02_l2/sq.log 2>&1
echo rc=$?
python - <<'PY'
import csv, collections
def agg(path):
    d = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"][:60]
        d[k][r["Counter_Name"]] += float(r["Counter_Value"])
    return d
for f in ["hit", "fetch", "sq"]:
    try:
        d = agg(f"gpurun_out/r02_l2/{f}/p_counter_collection.csv")
    except Exception as e:
        print(f, "missing", e); continue
    for k, v in d.items():
        if "gemm" in k: print(f, k, {a: round(b) for a, b in v.items()})
PY
python tools/prof_summary.py gpurun_out/r02_l2/trace/t_kernel_trace.csv --top 8
