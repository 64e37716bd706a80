"""Summarise an RC_RESOLVE_TRACE per-segment trace: when each segment starts/ends (10 ns
ticks of s_memrealtime), which segments end last, team rounds.
  python scripts/seg_trace.py TRACE"""
import sys
path = sys.argv[1]
seg = {}
for l in open(path):
    if l.startswith("#"):
        continue
    k, start, ln, ticks, evals, cyc = map(int, l.split())
    seg[k] = dict(start=start, len=ln, dur=ticks, evals=evals, cyc=cyc)
for l in open(path + ".start"):
    k, t = map(int, l.split())
    if k in seg:
        seg[k]["t0"] = t
team = [k for k, d in seg.items() if d["evals"] & 0x80000000]
t0s = [d["t0"] for k, d in seg.items() if k not in team and d.get("t0")]
base = min(t0s) if t0s else 0
ends = []
for k, d in seg.items():
    if k in team:
        continue
    t = (d.get("t0", base) - base) & 0xffffffff
    ends.append(((t + d["dur"]) / 100.0, t / 100.0, d["dur"] / 100.0, d["len"], d["evals"], k))
ends.sort(reverse=True)
print("segments:", len(seg), "team:", len(team), "total entries:", sum(d["len"] for d in seg.values()))
for k in team:
    d = seg[k]
    print(f"team seg {k}: len {d['len']} dur {d['dur']/100:.1f} us rounds {d['evals'] & 0x7fffffff}")
print("last-ending regular segments (end_us start_us dur_us len evals seg):")
for e in ends[:15]:
    print("  %.1f %.1f %.1f %d %d %d" % e)
busy = sum(d["dur"] for k, d in seg.items() if k not in team) / 100.0
print(f"regular wave-time: {busy/1000:.1f} wave-ms; longest 10 durations (us):",
      sorted((d["dur"] / 100 for k, d in seg.items() if k not in team), reverse=True)[:10])

import os
if os.path.exists(path + ".waves"):
    we = {}
    for l in open(path + ".waves"):
        k, t = map(int, l.split())
        we[k] = ((t - base) & 0xffffffff) / 100.0
    last = sorted(we.items(), key=lambda kv: -kv[1])[:12]
    print("last waves to leave (block*4+wave: us):", ", ".join(f"{k}: {v:.0f}" for k, v in last))
for k in team:
    d = seg[k]
    if d.get("t0"):
        print(f"team seg {k} starts at {(((d['t0'] - base + 2**31) & 0xffffffff) - 2**31) / 100:.1f} us")
if os.path.exists(path + ".cyc"):   # helper items (dense runs handed off by regular waves)
    for l in open(path + ".cyc"):
        if not l.startswith("item"):
            continue
        f = l.split()
        d = dict(zip(f[0::2], f[1::2]))
        s = int(d["seg"])
        t0 = ((int(d["t0"]) - base) & 0xffffffff) / 100.0
        t1 = ((int(d["t1"]) - base) & 0xffffffff) / 100.0
        st = ((seg[s].get("t0", base) - base) & 0xffffffff) / 100.0 if s in seg else float("nan")
        print(f"helper item {d['item']}: seg {s} len {seg[s]['len'] if s in seg else '?'} "
              f"seg start {st:.0f} us, handed off {t0:.0f} us, done {t1:.0f} us, "
              f"{d['changers']} changers in {d['coop']} cooperative steps")
