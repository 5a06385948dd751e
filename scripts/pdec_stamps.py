"""Explain the persistent decoder pass (k_pdec.hip) edge by edge from its per-unit stage stamps.

Input: the SPT_PD_STAMP file of one pass (u64 [CUs][kPdStampMax=512][10], 100 MHz s_memrealtime):
record = {meta = l | s << 8 | u << 16, gather start, gather wave 0 inputs ready, compute after barrier
A, compute weights landed, gather after barrier B, compute done, publish landed, compute after the
next unit's prefetch issue, compute after barrier B} (r6c files: the first 8 fields only).

Per layer the stages run in dependency order (A: LN1 + QKV, B: self-attention, C: self-out, D: LN2 +
cross-Q, E: cross-attention, E2: merge, F: cross-out, G: LN3 + fc1, H: fc2).  A stage's share of the
layer is last_publish(stage) - last_publish(previous stage); for the unit that published last, that
share is split into
  edge      previous stage's last publish -> this unit's inputs ready (gather wave 0 poll done)
  barrierA  inputs ready -> compute waves past barrier A (the other gather waves, the unit before)
  weights   barrier A -> this unit's prefetched operands landed
  compute   weights landed -> compute done
  barrierB  compute done -> gather wave 0 past barrier B
  publish   -> output granules landed (s_waitcnt vmcnt(0) after the stores)
usage: python3 scripts/pdec_stamps.py STAMPFILE [label]"""
import sys

import numpy as np

STAGES = ["A qkv", "B self-attn", "C self-out", "D cross-q", "E cross-attn", "E2 merge", "F cross-out", "G fc1",
          "H fc2"]
# guide rows (MI355X_MICROARCH.md, persistent kernels price list) for each stage's input edge
GUIDE = {0: "allgather (x rows, LN) 4.0-4.2", 1: "handoff-1to1 1.5-2.9", 2: "allgather 4.0-4.2",
         3: "allgather (x rows, LN) 4.2", 4: "handoff-1to1 1.5-2.9", 5: "handoff-1to1 (8 partials) 1.5-2.9",
         6: "allgather 4.0-4.2", 7: "allgather (x rows, LN) 4.2", 8: "allgather + payload > 32 KB 4.2 + >=4"}


def main():
    path = sys.argv[1]
    label = sys.argv[2] if len(sys.argv) > 2 else path
    raw = np.fromfile(path, dtype=np.uint64)
    nf = 10 if raw.size % (512 * 10) == 0 else 8  # r6c files hold 8 fields per record
    a = raw.reshape(-1, 512, nf).astype(np.int64)
    ncu = a.shape[0]
    rec = a.reshape(-1, nf)
    rec = rec[rec[:, 1] != 0]
    meta = rec[:, 0]
    l, s, u = meta & 0xFF, (meta >> 8) & 0xFF, meta >> 16
    L = int(l.max()) + 1
    t0 = rec[:, 1:].min()
    t = (rec[:, 1:] - t0) / 100.0  # us
    g_start, g_ready, c_a, c_w, g_b, c_done, pub = (t[:, i] for i in range(7))
    c_pf = t[:, 7] if nf == 10 else c_done
    c_b = t[:, 8] if nf == 10 else g_b
    last_pub = np.zeros((L, 9))
    crit = {}
    for li in range(L):
        for si in range(9):
            m = (l == li) & (s == si)
            if not m.any():
                last_pub[li, si] = np.nan
                continue
            idx = np.where(m)[0]
            k = idx[np.argmax(pub[idx])]
            last_pub[li, si] = pub[k]
            crit[(li, si)] = (k, int(m.sum()))
    rows = []
    for li in range(L):
        for si in range(9):
            if (li, si) not in crit:
                continue
            k, n = crit[(li, si)]
            prev = last_pub[li, si - 1] if si > 0 else (last_pub[li - 1, 8] if li > 0 else 0.0)
            rows.append((li, si, n, last_pub[li, si] - prev, g_ready[k] - prev, c_a[k] - g_ready[k], c_w[k] - c_a[k],
                         c_done[k] - c_w[k], g_b[k] - c_done[k], pub[k] - g_b[k], c_pf[k] - c_done[k], c_b[k] - c_pf[k]))
    R = np.array(rows)
    out = [f"# {label}: persistent decoder pass stage stamps ({ncu} workgroups, {L} layers, pass "
           f"{last_pub[L - 1, 8]:.1f} us from the first gather start = {last_pub[L - 1, 8] / L:.1f} us per layer)",
           "# per-stage share of the layer (last publish to last publish) and its split for the unit that published "
           "last; us, mean over layers 1..L-1 (layer 0 reads plain rows)",
           f"{'stage':<14}{'units':>6}{'share':>8}{'edge':>8}{'barA':>8}{'weights':>8}{'compute':>8}{'barB':>8}"
           f"{'publish':>8}{'[pf-iss':>8}{'barB-c]':>8}   guide row for the edge (us)",
           "# [pf-iss, barB-c]: the compute wave's part of barB -- issuing the next unit's prefetch, then waiting at B"]
    body = R[R[:, 0] >= 1] if L > 1 else R
    tot = np.zeros(9)
    for si in range(9):
        m = body[:, 1] == si
        if not m.any():
            continue
        v = body[m][:, 3:].mean(axis=0)
        tot += v
        out.append(f"{STAGES[si]:<14}{int(body[m][0, 2]):>6}" + "".join(f"{x:>8.2f}" for x in v) + f"   {GUIDE[si]}")
    out.append(f"{'layer':<14}{'':>6}" + "".join(f"{x:>8.2f}" for x in tot))
    # distribution of the inputs-ready time over a stage's units relative to the previous stage's last
    # publish (how long the last consumer waits after the first is already running)
    out.append("# consumer spread: inputs ready (gather wave 0) over all units of the stage, relative to the previous "
               "stage's last publish: min / median / max (mean over layers 1..L-1)")
    for si in range(9):
        v = []
        for li in range(1, L):
            m = (l == li) & (s == si)
            if not m.any():
                continue
            prev = last_pub[li, si - 1] if si > 0 else last_pub[li - 1, 8]
            r = g_ready[m] - prev
            v.append((r.min(), np.median(r), r.max()))
        if v:
            v = np.array(v).mean(axis=0)
            out.append(f"{STAGES[si]:<14}" + "".join(f"{x:>8.2f}" for x in v))
    print("\n".join(out))


if __name__ == "__main__":
    main()
