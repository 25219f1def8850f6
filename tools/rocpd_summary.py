#!/usr/bin/env python3
"""Summarise rocprofv3 SQLite output (ROCm 7.x `*_results.db`) into the files committed under profiles/.

  python tools/rocpd_summary.py stats  <kernel-trace .db>  <out.txt>
      per-kernel calls / total / average (microseconds) / share (the `--stats` kernel summary)
  python tools/rocpd_summary.py pmc    <kernel substring> <out.json> <pmc .db> [<pmc .db> ...]
      FETCH_SIZE / WRITE_SIZE of one kernel, one counter per pass (the two do not fit one pass on gfx950,
      MI355X_MICROARCH.md "rocprofv3 PMC slots") -> HBM bytes per launch

FETCH_SIZE and WRITE_SIZE are kilobytes (the counter description says so; x1024).  MI355X_MICROARCH.md
(HBM section): on gfx950 FETCH_SIZE reports 1/2 of the bytes of wide coalesced reads, so the corrected
fetch is 2 x FETCH_SIZE x 1024; WRITE_SIZE is taken as is.  Both are recorded.
"""
import json
import sqlite3
import sys


def stats(db, out):
    c = sqlite3.connect(db)
    rows = c.execute("select name, total_calls, total_duration, average, percentage from top_kernels").fetchall()
    # the rocpd `top_kernels` view reports (end - start) / 1000, i.e. microseconds
    lines = ["# rocprofv3 --kernel-trace --stats summary (%s)" % db,
             "# %-90s %8s %16s %14s %8s" % ("kernel", "calls", "total_us", "avg_us", "pct")]
    for name, calls, tot, avg, pct in rows:
        lines.append("%-92s %8d %16.1f %14.1f %8.3f" % (name[:92], calls, tot, avg, pct))
    open(out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def pmc(kernel, out, dbs):
    q = ("select dispatch_id, kernel_name, counter_name, value, duration from counters_collection "
         "where kernel_name like ? order by dispatch_id")
    totals, launches, per = {}, {}, []
    for db in dbs:
        c = sqlite3.connect(db)
        seen = set()
        for did, name, cname, value, dur in c.execute(q, ("%" + kernel + "%",)):
            totals[cname] = totals.get(cname, 0.0) + value
            seen.add(did)
            per.append({"db": db, "dispatch": did, "counter": cname, "value": value, "duration_ns": dur})
        for cname in {p["counter"] for p in per if p["db"] == db}:
            launches[cname] = len(seen)
    fetch_kb = totals.get("FETCH_SIZE", 0.0)
    write_kb = totals.get("WRITE_SIZE", 0.0)
    nf = max(launches.get("FETCH_SIZE", 1), 1)
    nw = max(launches.get("WRITE_SIZE", 1), 1)
    res = {
        "sources": dbs, "kernel": kernel, "launches": launches,
        "fetch_size_kb_total": fetch_kb, "write_size_kb_total": write_kb,
        "fetch_bytes_per_launch": 2.0 * fetch_kb * 1024.0 / nf,
        "write_bytes_per_launch": write_kb * 1024.0 / nw,
        "hbm_bytes_per_launch": 2.0 * fetch_kb * 1024.0 / nf + write_kb * 1024.0 / nw,
        "correction": "FETCH_SIZE (KB) x1024 x2 (gfx950 half-count, MI355X_MICROARCH.md HBM section); WRITE_SIZE x1024",
        # every collected counter per launch (raw units; see the correction above for FETCH_SIZE)
        "per_launch": {k: v / max(launches.get(k, 1), 1) for k, v in totals.items()},
        "per_dispatch": per,
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k: v for k, v in res.items() if k != "per_dispatch"}, indent=1))


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    else:
        pmc(sys.argv[2], sys.argv[3], sys.argv[4:])
