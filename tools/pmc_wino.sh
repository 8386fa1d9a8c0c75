# Investigative PMC passes (L2 hit rate / busy, LDS conflicts, instruction mix) over
# configs[2]; summarised on the box per kernel.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
ARGS="--model 3 --batch 256 --no-cpu-baseline --steps 3 --warmup 1 --profile-iters 1 --tune-step 0"
timeout -s KILL 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_BUSY_avr GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $R/gpurun_out/pw_a -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/pw_a.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_VALU_MFMA_F SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD --kernel-trace --output-format csv -d $R/gpurun_out/pw_b -o p -- python3 $R/bench.py $ARGS > $R/gpurun_out/pw_b.log 2>&1
python3 - <<'PY' > $R/gpurun_out/pmc_wino.txt
import csv, statistics, collections, os
R = os.environ.get("GRAFT_REPO_ROOT", ".")
vals = collections.defaultdict(lambda: collections.defaultdict(list))
durs = collections.defaultdict(list)
for d in ("pw_a", "pw_b"):
    p = f"{R}/gpurun_out/{d}/p_counter_collection.csv"
    seen = set()
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if "tic::" not in k:
            continue
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if (d, r["Dispatch_Id"]) not in seen:
            seen.add((d, r["Dispatch_Id"]))
            durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k in sorted(vals, key=lambda k: -statistics.median(durs[k]) * len(durs[k]))[:12]:
    v = {c: statistics.median(x) for c, x in vals[k].items()}
    hit = v.get("TCC_HIT_sum", 0); miss = v.get("TCC_MISS_sum", 0)
    print(k[:100])
    print("   us %.1f  L2 req %.3g hit%% %.1f  L2busy %.3g  lds_insts %.3g bankconf %.3g waitLDS %.3g valu %.3g mfma %.3g vmem_rd %.3g busy %.3g wavecyc %.3g" % (
        statistics.median(durs[k]), hit + miss, 100 * hit / max(1, hit + miss), v.get("TCC_BUSY_avr", 0),
        v.get("SQ_INSTS_LDS", 0), v.get("SQ_LDS_BANK_CONFLICT", 0), v.get("SQ_WAIT_INST_LDS", 0),
        v.get("SQ_INSTS_VALU", 0), v.get("SQ_INSTS_VALU_MFMA_F", 0), v.get("SQ_INSTS_VMEM_RD", 0),
        v.get("SQ_BUSY_CYCLES", 0), v.get("SQ_WAVE_CYCLES", 0)))
PY
rm -rf $R/gpurun_out/pw_a $R/gpurun_out/pw_b
