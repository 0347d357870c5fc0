"""Would per-lane band windows make the lane engine (csrc/ksw_lane.h) compute
fewer cells?  A model of one 64-lane wave running ksw_extend2 problems
(software/ksw.c:379-476) one per lane, on the row bands [beg, end) the
reference's own row loop produces (tools/ksw_bands.py's restatement), over
problems shaped like mem_chain2aln's (synth.make_ksw_tasks), sorted by query
length as the engine's queues sort them.  CPU only.

Per wave row it counts the 8-column chunks the engine runs:
  union    -- the engine as built: a chunk runs when any live lane's band
              (or end column) touches it (absolute columns in registers);
  per-lane -- a window that slides with each lane's own band: a row costs
              the widest band's chunk count among the live lanes;
and the in-band cells the reference computes, for lane-refill policies
REFILL = 8 (the engine's), 32, 64 (lockstep).

    python tools/ksw_band_sim.py [--problems 600] [--min-qlen 65] [--max-qlen 128]

Round 4 result (profiles/r04/ksw/band_sim.txt): the two counts are equal --
at any wave row some live lane is in its early rows, whose band spans the
whole query (beg stays 0 while the first column's H is positive, and end
reaches the query end), so a per-lane window buys nothing; lockstep refills
lose more to idle lanes than they gain.
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bwa-mem-harp2_amd"))
sys.path.insert(0, ROOT)


def bands_of(q, t, w, end_bonus, zdrop, h0, mat, o_del=6, e_del=1, o_ins=6, e_ins=1):
    """ksw_extend2's row loop (software/ksw.c:379-476), returning each row's
    band [beg, end) -- a plain restatement, top = 1 (mat's largest score)."""
    qlen, tlen = len(q), len(t)
    oe_del, oe_ins = o_del + e_del, o_ins + e_ins
    h, e = [0] * (qlen + 1), [0] * (qlen + 1)
    h0 = max(h0, 0)
    h[0] = h0
    h[1] = h0 - oe_ins if h0 > oe_ins else 0
    j = 2
    while j <= qlen and h[j - 1] > e_ins:
        h[j] = h[j - 1] - e_ins
        j += 1
    mi = max(int((qlen + end_bonus - o_ins) / e_ins + 1.), 1)
    w = min(w, mi)
    md = max(int((qlen + end_bonus - o_del) / e_del + 1.), 1)
    w = min(w, md)
    mx, max_i, max_j, beg, end, out = h0, -1, -1, 0, qlen, []
    for i in range(tlen):
        f, m, mj = 0, 0, -1
        h1 = max(h0 - (o_del + e_del * (i + 1)), 0)
        beg = max(beg, i - w)
        end = min(end, i + w + 1, qlen)
        out.append((beg, end))
        for jj in range(beg, end):
            M, E = h[jj], e[jj]
            h[jj] = h1
            M += mat[t[i]][q[jj]]
            H = max(M, E, f)
            h1 = H
            if H >= m:
                mj, m = jj, H
            E = max(E - e_del, max(H - oe_del, 0))
            e[jj] = E
            f = max(f - e_ins, max(H - oe_ins, 0))
        h[end], e[end] = h1, 0
        if m == 0:
            break
        if m > mx:
            mx, max_i, max_j = m, i, mj
        elif zdrop > 0:
            if i - max_i > mj - max_j:
                if mx - m - ((i - max_i) - (mj - max_j)) * e_del > zdrop:
                    break
            elif mx - m - ((mj - max_j) - (i - max_i)) * e_ins > zdrop:
                break
        jj = mj
        while jj >= beg and h[jj]:
            jj -= 1
        beg = jj + 1
        jj = mj + 2
        while jj <= end and h[jj]:
            jj += 1
        end = jj
    return out


def simulate(probs, refill, per_lane, nlanes=64, nchunks=16):
    lanes = [None] * nlanes
    qi = rows = chunks = inband = lane_rows = 0
    while True:
        idle = [l for l in range(nlanes) if lanes[l] is None]
        if idle and (len(idle) >= refill or len(idle) == nlanes):
            for l in idle:
                if qi < len(probs):
                    lanes[l] = [qi, 0]
                    qi += 1
        live = [l for l in range(nlanes) if lanes[l] is not None]
        if not live:
            break
        rows += 1
        used, widest = set(), 0
        for l in live:
            p, r = lanes[l]
            bg, en = probs[p][1][r]
            inband += max(en - bg, 0)
            lane_rows += 1
            for c in range(nchunks):
                if 8 * c <= en and 8 * c + 8 > min(bg, en):
                    used.add(c)
            widest = max(widest, (en + 8) // 8 - bg // 8)
        chunks += widest if per_lane else len(used)
        for l in live:
            lanes[l][1] += 1
            if lanes[l][1] >= len(probs[lanes[l][0]][1]):
                lanes[l] = None
    return rows, chunks, inband, lane_rows


def main():
    import numpy as np
    from smemgpu import synth
    ap = argparse.ArgumentParser()
    ap.add_argument("--problems", type=int, default=600)
    ap.add_argument("--min-qlen", type=int, default=65)
    ap.add_argument("--max-qlen", type=int, default=128)
    a = ap.parse_args()
    g = synth.make_genome(2_000_000, seed=771, n_chrom=1)
    kb = synth.make_ksw_tasks(g.codes, 3000, seed=771)
    mat = np.array(kb.mat, dtype=np.int64).reshape(5, 5)
    sel = [k for k in range(kb.tasks.size) if a.min_qlen <= kb.tasks["qlen"][k] <= a.max_qlen][:a.problems]
    probs = []
    for k in sel:
        T = kb.tasks[k]
        qo, to = int(T["q_off"]), int(T["t_off"])
        q, t = kb.q[qo:qo + int(T["qlen"])], kb.t[to:to + int(T["tlen"])]
        b = bands_of(list(q), list(t), int(T["w"]), int(T["end_bonus"]), int(T["zdrop"]), int(T["h0"]), mat)
        if b:
            probs.append((int(T["qlen"]), b))
    probs.sort(key=lambda p: p[0])
    print(f"{len(probs)} problems, query length {a.min_qlen}-{a.max_qlen} (the 128-column tier)")
    for refill in (8, 32, 64):
        for per_lane in (False, True):
            w, c, ib, lr = simulate(probs, refill, per_lane)
            print(f"refill {refill:2d} {'per-lane' if per_lane else 'union':8s}: wave rows {w}, live lanes/row "
                  f"{lr / w:.1f}, chunks/row {c / w:.1f}, in-band / computed lane-cells {ib / (c * 8 * 64):.3f}")


if __name__ == "__main__":
    main()
