cd $GRAFT_REPO_ROOT
O=gpurun_out/r02n; mkdir -p $O
export TMPDIR=/tmp
for v in x_base x_w16 x_w16w3 x_basew3; do
  echo "== $v"
  AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so timeout -k 10 150 python tools/k5_probe.py 8388608 2>&1 | tail -3 || exit 1
done
for v in x_base x_w16 x_w16w3 x_basew3; do
  export AVDB_LIB=annotatedvdb_amd/_lib/var/libavdb_$v.so
done
python3 - $O <<'PY'
import csv, glob, sys, collections
for d in sorted(glob.glob(sys.argv[1] + "/w_*/")):
    fs = glob.glob(d + "**/*counter_collection.csv", recursive=True)
    tot = collections.defaultdict(list)
    for r in csv.DictReader(open(fs[0])):
        if "k_vcf_format" in r["Kernel_Name"]:
            k = ("W " if "<true>" in r["Kernel_Name"] else "S ") + r["Counter_Name"]
            tot[k].append(float(r["Counter_Value"]))
    print(d, {k: "%.4g" % (sum(v) / len(v)) for k, v in tot.items()})
PY
