"""Per-frame timeline of frames in flight from a rocprofv3 kernel trace: phase A, compaction,
resolver and phase C start / end of every frame (ms from the 4th frame's phase A), its lane and
slot, and the gap between a lane's resolver end and the next kernel that waits on it.
   python3 scripts/pipe_frames.py TRACE.csv"""
import csv, sys
rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rc::", "").split("<")[0]
    if n.startswith("k_"):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, int(r["Correlation_Id"])))
rows.sort(key=lambda x: x[3])
fr, cur = [], None
for s, e, n, c in rows:
    if n == "k_phase_a":
        cur = {"A": (s, e)}
        fr.append(cur)
    elif cur is not None:
        cur.setdefault(n, (s, e))
t0 = fr[3]["A"][0]
print("frame   A_start  A_end comp_end  R_start  R_end  C_start  C_end  R->C gap")
for i, f in enumerate(fr[3:], 3):
    g = lambda k, j: (f[k][j] - t0) / 1e6 if k in f else float("nan")
    print("%3d  %7.2f %7.2f %7.2f  %7.2f %7.2f  %7.2f %7.2f  %6.2f  lane %d" % (
        i, g("A", 0), g("A", 1), g("k_seg_order", 1), g("k_resolve", 0), g("k_resolve", 1),
        g("k_dep_chunks", 0), g("k_dep_chunks", 1), g("k_dep_chunks", 0) - g("k_resolve", 1), i % 2))
