cd $GRAFT_REPO_ROOT && export TMPDIR=/tmp && mkdir -p gpurun_out
for k in 1 4; do
COA_CERT_K=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS -d gpurun_out/pmc_cert$k -o run --output-format csv -- python3 tools/cert_probe.py 10000 > gpurun_out/pmc_cert$k.log 2>&1 || exit 1
f=$(find gpurun_out/pmc_cert$k -name "*counter_collection.csv" | head -1)
python3 - "$f" $k <<'PY'
import csv,sys,collections
rows=list(csv.DictReader(open(sys.argv[1])))
agg=collections.defaultdict(lambda: collections.defaultdict(float)); n=collections.Counter()
for r in rows:
    k=r["Kernel_Name"].split('(')[0]
    if 'k_cert_verify<' not in r["Kernel_Name"] and 'k_cert_verifyILi' not in r["Kernel_Name"]: continue
    agg[k][r["Counter_Name"]]+=float(r["Counter_Value"])
for k,v in agg.items():
    w=v["SQ_WAVES"]; print("K=",sys.argv[2],k[:60], {c: round(x/w,1) for c,x in v.items()}, "wait_any/wave_cycles", round(v["SQ_WAIT_ANY"]/v["SQ_WAVE_CYCLES"],3), "wait_inst/wave_cycles", round(v["SQ_WAIT_INST_ANY"]/v["SQ_WAVE_CYCLES"],3))
PY
done
