cd $GRAFT_REPO_ROOT
O=gpurun_out/r02l; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || timeout -k 10 120 rocprofv3 --list-avail > $O/counters.txt 2>&1
grep -oE "(TA|TD|TCP|TCC|SQ|GRBM)_[A-Z0-9_]+" $O/counters.txt | sort -u > $O/names.txt
wc -l $O/names.txt
grep -E "^(TA|TD|TCP)_" $O/names.txt | tr '\n' ' '
