cd $GRAFT_REPO_ROOT
O=gpurun_out/r02m; mkdir -p $O
export TMPDIR=/tmp
for v in t0 t1_disp; do
  echo "== $v"
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 150 python tools/k5_probe.py 8388608 2>&1 | grep -v checksum | tail -2 || exit 1
done
exit 0
timeout -s KILL 120 rocprofv3 --pmc TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE -d $O/p1 -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_WRITE_TAGCONFLICT_STALL_CYCLES_sum -d $O/p2 -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/p2.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY_sum TD_TC_STALL_sum -d $O/p3 -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/p3.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
for d in sorted(glob.glob(sys.argv[1] + "/p*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs: continue
    tot = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        if "k_vcf_format" in r["Kernel_Name"]:
            k = ("W " if "<true>" in r["Kernel_Name"] else "S ") + r["Counter_Name"]
            tot[k].append(float(r["Counter_Value"]))
    print(d)
    for k, v in sorted(tot.items()):
        print("  %-40s %.4g" % (k, sum(v) / len(v)))
PY
