cd $GRAFT_REPO_ROOT
bash tools/traffic_counters.sh c2 r02q/c2 || exit 1
bash tools/traffic_counters.sh c5 r02q/c5 || exit 1
bash tools/traffic_counters.sh load r02q/load || exit 1
