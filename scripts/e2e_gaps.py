"""Line up scripts/e2e_trace_run.py's calls with a rocprofv3 kernel + HIP API trace: per call,
the kernels (start/end in ms from the call's start), the calling thread's HIP API calls, and
the device's idle time before its first kernel and after its last.
Usage: python scripts/e2e_gaps.py RUN_LOG TRACE_DIR [call]"""
import csv
import glob
import os
import re
import sys

log, tdir = sys.argv[1], sys.argv[2]
only = int(sys.argv[3]) if len(sys.argv) > 3 else None
calls = []
for line in open(log):
    m = re.match(r"call (\d+) start_ns (\d+) end_ns (\d+)", line)
    if m:
        calls.append((int(m.group(1)), int(m.group(2)), int(m.group(3))))
kern = list(csv.DictReader(open(glob.glob(os.path.join(tdir, "*kernel_trace.csv"))[0])))
api = list(csv.DictReader(open(glob.glob(os.path.join(tdir, "*hip_api_trace.csv"))[0])))
main_tid = api[0]["Process_Id"]
for i, t0, t1 in calls:
    if only is not None and i != only:
        continue
    ks = sorted((int(k["Start_Timestamp"]), int(k["End_Timestamp"]), k["Kernel_Name"][:40])
                for k in kern if t0 <= int(k["Start_Timestamp"]) <= t1)
    ms = lambda t: (t - t0) / 1e6
    print(f"call {i}: {ms(t1):.3f} ms; device first kernel at {ms(ks[0][0]):.3f}, last ends "
          f"{ms(ks[-1][1]):.3f} (idle after it {ms(t1) - ms(ks[-1][1]):.3f} ms)")
    if only is None:
        continue
    for a, b, n in ks:
        print(f"  K {ms(a):8.3f} {ms(b):8.3f}  {n}")
    for r in api:
        if r["Thread_Id"] != main_tid:
            continue
        a, b = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if t0 <= a <= t1:
            print(f"  A {ms(a):8.3f} {ms(b):8.3f}  {r['Function']}")
