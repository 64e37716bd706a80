"""Dense-run carry prediction, simulated on the CPU oracle's exact carries (no GPU).

The resolver's predictive steps (rc_kernels.hip: wave_window, block_window with a CarryHist)
evaluate entry pos at the exact carry and entry pos+1 (and, with RC_PRED_SPLIT, pos+2) at
guessed carry-ins bits(c) + k * mean delta of the last changes (+-1, +-2 .. ulps on the moving
component); a guess that equals the exact output retires the next entry in the same step.
This replays that rule on the oracle's carry-in sequence (scripts/pred_dump.py writes it) for
every dense segment (> 200 entries, > 50 % changers) and prints entries retired per step for
splits (k1 guesses for pos+1, k2 for pos+2): 3/0 is a regular wave, 15/0 a helper block.
   python3 scripts/pred_dump.py 4096 && python3 scripts/pred_sim.py
"""
import numpy as np

cb = np.load("/tmp/carries.npy")
starts, lens = np.load("/tmp/segs.npy")


def md_of(h):   # mean step of the history h (latest first), hist_guess's rounding
    m = len(h) - 1
    d = h[0] - h[m]
    if m == 1:
        return d
    q = d + np.where(d >= 0, 1, -1)
    return np.where(q >= 0, q // m, -((-q) // m))


def guesses(c, md, mult, k):
    g = c + mult * md
    a = np.abs(md)
    mv = 0 if (a[0] >= a[1] and a[0] >= a[2]) else (1 if a[1] >= a[2] else 2)
    out = []
    for j in range(k):
        x = g.copy()
        x[mv] += (-((j + 1) >> 1)) if (j & 1) else (j >> 1)
        out.append(x)
    return out


def steps(lo, hi, k1, k2):
    pos, n, hist = lo, 0, []
    while pos < hi - 1:
        c = cb[pos]
        n += 1
        o0 = cb[pos + 1]
        if len(hist) < 2:
            hist = ([o0] + (hist or [c]))[:4] if (o0 != c).any() else []
            pos += 1
            continue
        md = md_of(hist)
        if (o0 == c).all():
            hist, pos = [], pos + 1
            continue
        if pos + 2 >= hi or not any((g == o0).all() for g in guesses(c, md, 1, k1)):
            hist, pos = ([o0] + hist)[:4], pos + 1
            continue
        o1 = cb[pos + 2]
        if (o1 == o0).all():
            hist, pos = [], pos + 2
            continue
        if k2 and pos + 3 < hi and any((g == o1).all() for g in guesses(c, md, 2, k2)):
            o2 = cb[pos + 3]
            hist = ([o2, o1, o0] + hist)[:4] if (o2 != o1).any() else []
            pos += 3
        else:
            hist, pos = ([o1, o0] + hist)[:4], pos + 2
    return n


ch = np.any(cb[1:] != cb[:-1], axis=1)
dense = [(s, l) for s, l in zip(starts, lens) if l > 200 and ch[s:s + l - 1].mean() > 0.5]
print("dense segments (length):", [int(l) for _, l in dense])
for k1, k2 in [(3, 0), (2, 1), (15, 0), (7, 8), (9, 6), (11, 4)]:
    print(f"{k1:2d}/{k2:<2d}", [round(float(l) / steps(s, s + l, k1, k2), 2) for s, l in dense])
