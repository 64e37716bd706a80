"""Per-kernel register / scratch / occupancy table of a HIP source (hipcc
-Rpass-analysis=kernel-resource-usage), for before/after comparisons of a kernel change.
   python3 scripts/res_usage.py [SRC] [extra hipcc flags...]"""
import re, subprocess, sys
src = sys.argv[1] if len(sys.argv) > 1 else "raytracing-programs_amd/csrc/rc_kernels.hip"
flags = ("--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off "
         "-fno-gpu-flush-denormals-to-zero -fhip-fp32-correctly-rounded-divide-sqrt "
         "-Iinclude -Iraytracing-programs_amd/csrc -w --cuda-device-only").split() + sys.argv[2:]
r = subprocess.run(["/opt/rocm/bin/hipcc", *flags, "-Rpass-analysis=kernel-resource-usage",
                    "-c", src, "-o", "/dev/null"], capture_output=True, text=True)
cur, rows = None, {}
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?) \[-Rpass", line)
    if not m:
        continue
    k, _, v = m.group(1).strip().partition(": ")
    if k == "Function Name":
        cur = v
        rows[cur] = {}
    elif cur:
        rows[cur][k] = v
for name, d in rows.items():
    short = re.sub(r"^_ZN2rc\d+", "", name)[:40]
    print(f"{short:40s} vgpr {d.get('VGPRs','?'):>4} agpr {d.get('AGPRs','?'):>3} "
          f"scratch {d.get('ScratchSize [bytes/lane]','?'):>4} occ {d.get('Occupancy [waves/SIMD]','?'):>2} "
          f"vspill {d.get('VGPRs Spill','?'):>3} lds {d.get('LDS Size [bytes/block]','?')}")
