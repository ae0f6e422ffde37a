import json, sys
rows = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
for r in rows:
    if "MISMATCH" in r:
        print("MISMATCH", r)
keys = sorted({(r["workload"], r["hist"]) for r in rows if "GBps" in r})
for wl, h in keys:
    rs = sorted([r for r in rows if r.get("workload") == wl and r.get("hist") == h and "GBps" in r], key=lambda r: -r["GBps"])
    print(wl, "hist" if h else "nohist")
    for r in rs[:6]:
        print("   ", {k: r[k] for k in r if k not in ("workload", "hist")})
    print("    worst", rs[-1]["GBps"])
