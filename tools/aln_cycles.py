"""Per-read shader cycles of chains -> regions (aln_prof.py --cycles dump:
u64 per read, written by the light walk and the heavy walk) beside each read's
chain / seed counts: the heaviest reads and the totals.

    python tools/aln_cycles.py <dump> [<dump> ...]
"""
import sys

import numpy as np

for f in sys.argv[1:]:
    cyc = np.fromfile(f, dtype=np.uint64).astype(np.float64)
    z = np.load(f + ".chains.npz")
    nch = np.diff(z["chain_off"].astype(np.int64))
    print(f, "reads", cyc.size, "total %.0f M cycles, mean %.0f k" % (cyc.sum() / 1e6, cyc.mean() / 1e3))
    for i in np.argsort(-cyc)[:12]:
        print("  read %d: %.1f M cycles, %d chains, %d bp" % (i, cyc[i] / 1e6, nch[i], z["lens"][i]))
    for lo, hi in [(0, 17), (17, 64), (64, 256), (256, 1024), (1024, 1 << 30)]:
        m = (nch >= lo) & (nch < hi)
        if m.any():
            print("  chains %d-%d: %d reads, max %.1f M cycles, sum %.0f M" % (lo, hi - 1, m.sum(), cyc[m].max() / 1e6,
                                                                            cyc[m].sum() / 1e6))
