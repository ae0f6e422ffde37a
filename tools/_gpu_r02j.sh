cd $GRAFT_REPO_ROOT
O=gpurun_out/r02j; mkdir -p $O
export TMPDIR=/tmp
for v in a_old e_sect36w3_t f_sect28w4_t; do
  echo "== $v"
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 150 python tools/k5_probe.py 8388608 || exit 1
done
for v in a_old e_sect36w3_t f_sect28w4_t; do
  export AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$v -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/pmcw_$v.log 2>&1 || exit 1
done
export AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_a_old.so
timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR -d $O/sq1_a -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/sq1_a.log 2>&1 || exit 1
timeout -s KILL 150 rocprofv3 --pmc SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM -d $O/sq2_a -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/sq2_a.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys, collections
for d in sorted(glob.glob(sys.argv[1] + "/*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    if not fs: continue
    tot = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        if "k_vcf_format" in r["Kernel_Name"]:
            k = ("W " if "<true>" in r["Kernel_Name"] else "S ") + r["Counter_Name"]
            tot[k].append(float(r["Counter_Value"]))
    print(d)
    for k, v in sorted(tot.items()):
        print("  %-28s %.4g" % (k, sum(v) / 4))
PY
