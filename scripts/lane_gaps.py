"""Why a resolver lane idles between its resolvers, from a rocprofv3 kernel
trace of the frames-in-flight bench (scripts/gpu_lane_trace.sh).  For each frame's k_resolve:
its lane (queue), the end of the lane's previous resolver, the end of the frame's compaction
(k_seg_order: the event the resolver waits on), and the start.  The lane's idle gap splits into
`comp_late` (the lane waited for this frame's compaction) and `dispatch` (the start after both
were done).  Frames are matched by order: the i-th k_resolve belongs to the i-th k_seg_order.
   python3 scripts/lane_gaps.py gpurun_out/<tag>_trace/k_kernel_trace.csv [frames]"""
import csv
import sys

rows = []
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("rc::", "").split("<")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), n, r["Queue_Id"]))
rows.sort()
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 20
res = [x for x in rows if x[2] == "k_resolve"]
seg = [x for x in rows if x[2] == "k_seg_order"]
pha = [x for x in rows if x[2] == "k_phase_a"]
assert len(res) == len(seg) == len(pha), (len(res), len(seg), len(pha))
first = len(res) - nf
last_end = {}
ms = lambda v: v / 1e6
print(f"{'frame':>5} {'lane':>4} {'gap':>6} {'comp_late':>9} {'dispatch':>8} {'phaseA_start_after_prev':>24} {'phaseA':>7} {'comp':>6}")
tot = {}
for i, (s, e, _, q) in enumerate(res):
    prev = last_end.get(q)
    last_end[q] = e
    if i < first or prev is None:
        continue
    ready = seg[i][1]
    gap = s - prev
    comp_late = max(0, ready - prev)
    disp = s - max(ready, prev)
    pa_s, pa_e = pha[i][0], pha[i][1]
    pa_prev_end = pha[i - 1][1] if i > 0 else pa_s
    print(f"{i:5d} {q:>4} {ms(gap):6.3f} {ms(comp_late):9.3f} {ms(disp):8.3f} {ms(pa_s - pa_prev_end):24.3f} "
          f"{ms(pa_e - pa_s):7.3f} {ms(ready - pa_e):6.3f}")
    t = tot.setdefault(q, [0, 0, 0, 0])
    t[0] += gap; t[1] += comp_late; t[2] += disp; t[3] += 1
for q, (g, c, d, n) in tot.items():
    print(f"lane queue {q}: {n} gaps, mean {ms(g) / n:.3f} ms = compaction late {ms(c) / n:.3f} + "
          f"dispatch {ms(d) / n:.3f}")
