"""Host study of the serial-equivalent (exact) training on the bench's stream:
how many samples of a batch could update, and how far the rest stay from
their threshold, under the bound the GPU committer verifies
(csrc/hip/commit.hip: a sample whose slack at the segment start exceeds
2 sum_f |x_f| R_f - R_f the summed step magnitudes of row f in the segment -
cannot update there).

Per batch (the model trained serially on the host, jb_cpu_serial.cpp):
updates, distinct rows written, the slack / bound quantiles, and for each
candidate threshold T the candidate count |{slack0 <= T}| and the
non-candidates the final bound does not clear.

Usage: python tools/exact_study.py [--batches 40] [--worst-case]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, default=40)
    ap.add_argument("--requests", type=int, default=1024)
    ap.add_argument("--per-request", type=int, default=128)
    ap.add_argument("--worst-case", action="store_true")
    ap.add_argument("--every", type=int, default=5, help="report every k-th batch")
    ap.add_argument("--windows", default="131072,32768,8192")
    a = ap.parse_args()
    import numpy as np
    import torch  # noqa: F401  (bench.FreshStream allocates through torch)
    import bench
    from jubatus_amd._native import native
    from jubatus_amd.fv_converter.converter import DatumToFvConverter
    from jubatus_amd.fv_converter.gpu_path import GpuRuleTable

    nat = native()
    args = argparse.Namespace(requests=a.requests, per_request=a.per_request, labels=16,
                              str_features=8, num_features=8)
    p_corr, vocab = (0.0, (1 << 31) - 1) if a.worst_case else (0.6, 100000)
    data = bench.FreshStream(nat, torch, False, args, 12345, a.batches, 8, p_corr, vocab)
    cfg = json.loads(json.dumps(bench.AROW_CONFIG))
    H = 1 << 20
    cfg["converter"]["hash_max_size"] = H
    conv = DatumToFvConverter(cfg["converter"])
    rt = GpuRuleTable(conv)
    hasher = nat.HostFvHasher(rt.srules, rt.n_srules, rt.nrules, rt.n_nrules, rt.blob, H)
    table = nat.LabelTable()
    for y in range(16):
        table.get_or_add(f"label{y}")
    LC = 16
    W = np.zeros((H, LC), np.float32)
    P = np.ones((H, LC), np.float32)
    active = np.ones(LC, np.uint8)
    g = 1e-4
    wins = [int(w) for w in a.windows.split(",")]
    for b, arena in enumerate(data.batches):
        rp, idx, val, lab = nat.cpu_hash_arena(hasher, arena.np.ctypes.data,
                                               np.asarray(arena.offs, np.int64),
                                               np.asarray(arena.lens, np.int64), table)
        n = len(lab)
        nf = np.diff(rp)
        report = b % a.every == 0 or b == a.batches - 1
        if report:
            # scores at the batch start (M0), margin, slack of AROW (threshold 1)
            seg = np.repeat(np.arange(n), nf)
            ok = idx >= 0
            s0 = np.zeros((n, LC), np.float32)
            np.add.at(s0, seg[ok], val[ok, None] * W[idx[ok]])
            sy = s0[np.arange(n), lab]
            other = s0.copy()
            other[np.arange(n), lab] = -np.inf
            best = other.max(axis=1)
            slack0 = sy - best - 1.0 - g * (1 + np.abs(sy) + np.abs(best))
        mag = np.zeros(len(idx), np.float32)
        upd, sec = nat.cpu_serial_train(5, 1.0, LC, rp, idx, val, lab, active, W.ctypes.data,
                                        P.ctypes.data, mag)
        if not report:
            continue
        updated = np.zeros(n, bool)
        updated[np.unique(seg[mag > 0])] = True
        rec = {"batch": b, "updates": int(upd), "update_frac": round(upd / n, 4),
               "train_s": round(sec, 3), "samples_per_s": round(n / sec)}
        # candidate rules on window [8192, 16384) with [0, 8192) as the previous
        # window: absolute T, the bound predicted from the previous window's
        # row steps (kappa x 2 sum |x| R_prev, floor f), and the oracle (the
        # window's own final bound) - candidates and not-cleared non-candidates
        def rbound(lo, hi):
            sl_ = slice(rp[lo], rp[hi])
            Rw = np.zeros(H, np.float32)
            m_ = mag[sl_] > 0
            np.add.at(Rw, idx[sl_][m_], mag[sl_][m_])
            return Rw
        lo, hi = 8192, 16384
        if n >= hi:
            Rp, Rc = rbound(0, lo), rbound(lo, hi)
            sl_ = slice(rp[lo], rp[hi])
            ax = np.abs(val[sl_])
            ok_ = idx[sl_] >= 0
            def bsum(R):
                return 2 * (1 + 4 * g) * np.add.reduceat(ax * np.where(ok_, R[np.maximum(idx[sl_], 0)], 0),
                                                         rp[lo:hi] - rp[lo])
            b_prev, b_true = bsum(Rp), bsum(Rc)
            s_ = slack0[lo:hi]
            rules = {}
            for T in (0.05, 0.125, 0.25):
                c_ = s_ <= T
                rules[f"abs{T}"] = (int(c_.sum()), int(((~c_) & (s_ <= b_true)).sum()))
            for kap in (1.0, 2.0, 4.0):
                for fl in (0.02, 0.05, 0.125):
                    c_ = s_ <= np.maximum(fl, kap * b_prev)
                    rules[f"prev_k{kap}_f{fl}"] = (int(c_.sum()), int(((~c_) & (s_ <= b_true)).sum()))
            c_ = s_ <= b_true
            rules["oracle"] = (int(c_.sum()), 0)
            rules["updates"] = int(updated[lo:hi].sum())
            rec["rules_w8192"] = rules
        for w in wins:
            # windows of w samples from the batch start: R over the window's updates
            lo, hi = 0, min(n, w)
            sl = slice(rp[lo], rp[hi])
            R = np.zeros(H, np.float32)
            np.add.at(R, idx[sl][mag[sl] > 0], mag[sl][mag[sl] > 0])
            xs = np.abs(val[sl]) * np.where(idx[sl] >= 0, R[np.maximum(idx[sl], 0)], 0)
            bound = 2 * (1 + 4 * g) * np.add.reduceat(xs, rp[lo:hi] - rp[lo]) if hi > lo else np.zeros(0)
            s = slack0[lo:hi]
            u = updated[lo:hi]
            rows = np.unique(idx[sl][mag[sl] > 0])
            wr = {"window": hi - lo, "updates": int(u.sum()), "rows_written": int(len(rows)),
                  "slack0_le0": int((s <= 0).sum()),
                  "bound_q": [float(np.quantile(bound, q)) for q in (0.5, 0.9, 0.99, 1.0)],
                  "not_cleared": int(((s <= bound) & ~(s <= 0)).sum())}
            for T in (0.0, 0.5, 1.0, 2.0, 4.0):
                cand = s <= T
                viol = (~cand) & (s <= bound)
                wr[f"T{T}"] = {"cand": int(cand.sum()), "viol": int(viol.sum()),
                               "first_viol": int(np.argmax(viol)) if viol.any() else None}
            rec[f"w{w}"] = wr
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
