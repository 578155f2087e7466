"""Per-work-group phase times of k_fused_v6 from its FRS_ANA_DBG records ("frs-wg block t_start t_p1 t_end tickets
last_ticket last_tile state tiles", s_memrealtime at 100 MHz): the last launch in the log, times in us from the
earliest start."""
import sys
import numpy as np

rows = [l.split()[1:] for l in open(sys.argv[1]) if l.startswith("frs-wg ")]
a = np.array([[int(x) for x in r] for r in rows], dtype=np.int64)
nwg = int(a[:, 0].max()) + 1
a = a[-nwg:]
for l in open(sys.argv[1]):
    if l.startswith("frs-fused"):
        last = l.strip()
print(last)
t0 = a[a[:, 1] > 0, 1].min()
rel = lambda c: (np.where(a[:, c] > 0, a[:, c] - t0, -1)) / 100.0
q = lambda v: " ".join(f"{x:8.1f}" for x in np.percentile(v, [0, 10, 50, 90, 100]))
print(f"work-groups {nwg}; percentiles 0/10/50/90/100 (us)")
print("start      ", q(rel(1)))
print("phase-1 end", q(rel(2)))
print("end        ", q(rel(3)))
print("tickets    ", q(a[:, 4].astype(float)))
print("tiles      ", q(a[:, 8].astype(float)))
states, counts = np.unique(a[:, 7], return_counts=True)
print("states", dict(zip(states.tolist(), counts.tolist())))
stuck = a[a[:, 7] != 4]
for r in stuck[:12]:
    print("not done: wg", r[0], "state", r[7], "ticket", r[5], "tile", r[6], "tickets", r[4], "tiles", r[8])
