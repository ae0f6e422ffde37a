cd $GRAFT_REPO_ROOT
O=gpurun_out/r02i; mkdir -p $O
export TMPDIR=/tmp
for v in a_old b_sect28w4 c_sect36w3 d_sect24w4; do
  echo "== $v"
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 150 python tools/k5_probe.py 8388608 || exit 1
done
for v in a_old b_sect28w4; do
  export AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so
  timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d $O/pmcw_$v -o run --output-format csv -- python3 tools/k5_probe.py 8388608 > $O/pmcw_$v.log 2>&1 || exit 1
  python3 - $O/pmcw_$v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
tot = {}
for r in csv.DictReader(open(f)):
    if "k_vcf_format" in r["Kernel_Name"]:
        k = r["Kernel_Name"].split("<")[1][:5]
        tot.setdefault(k, []).append(float(r["Counter_Value"]))
for k, v in tot.items():
    print(k, "launches", len(v), "WRITE_SIZE KiB/launch", sum(v) / len(v))
PY
done
