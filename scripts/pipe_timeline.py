"""Frames-in-flight timeline from a rocprofv3 kernel trace (scripts/pmc_headline.sh `stats`):
per kernel kind its busy time, and the pixel partition's utilisation — the union of the
intervals in which a pixel-partition kernel (phase A, compaction, phase C) runs — against the
resolver lanes' union, over the last N frames (the timed ones).
   python3 scripts/pipe_timeline.py gpurun_out/pmch/r04_stats/s_kernel_trace.csv [frames]"""
import csv, sys

path = sys.argv[1]
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 20
rows = []
for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rc::", "")
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n.split("<")[0]))
rows.sort()
res = [x for x in rows if x[2] == "k_resolve"]
t0 = res[-nf][0]   # the timed region: from the first timed frame's resolver on (approx.)
t1 = max(e for s, e, n in rows if n.startswith("k_"))


def union(iv):
    tot, cur_s, cur_e = 0, None, None
    for s, e in sorted(iv):
        s, e = max(s, t0), min(e, t1)
        if e <= s:
            continue
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                tot += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        tot += cur_e - cur_s
    return tot


span = t1 - t0
pix = [(s, e) for s, e, n in rows if n in ("k_phase_a", "k_dep_chunks")]
comp = [(s, e) for s, e, n in rows if n in ("k_row_stats", "k_row_scan", "k_row_compact", "k_seg_order")]
print(f"window {span / 1e6:.3f} ms ({nf} resolver launches from the end)")
print(f"pixel partition busy (phase A or phase C running): {union(pix) / span:.3f}")
print(f"  phase A running: {union([(s, e) for s, e, n in rows if n == 'k_phase_a']) / span:.3f}, "
      f"phase C running: {union([(s, e) for s, e, n in rows if n == 'k_dep_chunks']) / span:.3f}, "
      f"both: {(union([(s, e) for s, e, n in rows if n == 'k_phase_a']) + union([(s, e) for s, e, n in rows if n == 'k_dep_chunks']) - union(pix)) / span:.3f}")
print(f"compaction running: {union(comp) / span:.3f}")
print(f"some resolver running: {union([(s, e) for s, e, n in rows if n == 'k_resolve']) / span:.3f}")
# per lane (frames alternate between the two resolver streams)
rr = [(s, e) for s, e, n in rows if n == "k_resolve"]
for lane in (0, 1):
    iv = rr[lane::2]
    print(f"resolver lane {lane} busy: {union(iv) / span:.3f}")
gaps = []
for lane in (0, 1):
    iv = [x for x in rr[lane::2] if x[0] >= t0]
    gaps += [(iv[i + 1][0] - iv[i][1]) / 1e6 for i in range(len(iv) - 1)]
print("gaps between a lane's resolvers (ms): " + " ".join(f"{g:.2f}" for g in gaps))
pa = [(s, e) for s, e, n in rows if n == "k_phase_a" and s >= t0]
print("phase A durations (ms): " + " ".join(f"{(e - s) / 1e6:.2f}" for s, e in pa))
print("phase A start gaps after previous phase A end (ms): " + " ".join(f"{(pa[i + 1][0] - pa[i][1]) / 1e6:.2f}" for i in range(len(pa) - 1)))
