"""Summarise a diagnostic per-read cycle dump of the heavy-read walk (5 u64
arrays of n_reads: total, containment-scan, seed-order cycles, scans, scanned
chunks) beside the read's chain count; prints the heaviest reads and totals."""
import sys

import numpy as np

for f in sys.argv[1:]:
    c = np.fromfile(f, dtype=np.uint64).astype(np.float64)
    n = c.size // 5
    tot, scan, rank, nscan, nch = c[:n], c[n:2 * n], c[2 * n:3 * n], c[3 * n:4 * n], c[4 * n:]
    z = np.load(f + ".chains.npz")
    nchn = np.diff(z["chain_off"].astype(np.int64))
    h = np.where(scan + rank + nscan > 0)[0]
    print(f, "heavy reads walked", h.size)
    for i in h[np.argsort(-tot[h])][:8]:
        print("  read %d chains %d: total %.1fM cycles, scan %.1fM, order %.1fM, scans %d, chunks %d"
              % (i, nchn[i], tot[i] / 1e6, scan[i] / 1e6, rank[i] / 1e6, nscan[i], nch[i]))
    print("  sum: total %.0fM scan %.0fM order %.0fM" % (tot[h].sum() / 1e6, scan[h].sum() / 1e6, rank[h].sum() / 1e6))
