"""ctypes bindings of the HIP kernel library (csrc/hip/*.hip).

Every wrapper takes torch tensors that already live on the current HIP
device, checks shapes/dtypes on the host (a kernel never sees an operand it
was not written for), and launches on the current torch stream so kernels
order naturally with torch ops and RCCL collectives.
"""
from __future__ import annotations

import ctypes
import os
import time

import torch

from .._native import hip_lib
from ..utils import trace

_c_void_p = ctypes.c_void_p
_i32 = ctypes.c_int32
_i64 = ctypes.c_int64
_u64 = ctypes.c_uint64
_f32 = ctypes.c_float

_SIGS = {
    "jb_train_batch_submit": [_c_void_p],
    "jb_train_batch_args_bytes": [],
    "jb_event_create": [],
    "jb_event_destroy": [_i64],
    "jb_event_record": [_i64, _c_void_p],
    "jb_stream_wait_event": [_c_void_p, _i64],
    "jb_event_query": [_i64],
    "jb_event_sync": [_i64],
    "jb_fv_hash": [_c_void_p, _i64, _i64, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32,
                   _c_void_p, _i32, _c_void_p, _i32, _u64, _c_void_p, _c_void_p, _c_void_p,
                   _c_void_p],
    "jb_linear_train": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p,
                        _c_void_p, _c_void_p, _i32, _i32, _f32, _i32, _c_void_p, _c_void_p,
                        _c_void_p, _i32, _i32, _c_void_p, _c_void_p, _i64, _c_void_p, _i64,
                        _c_void_p],
    "jb_linear_train_bf16": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32,
                             _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _f32, _i32, _c_void_p,
                             _c_void_p, _c_void_p, _i64, _c_void_p],
    "jb_linear_classify_bf16": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32,
                                _c_void_p, _c_void_p],
    "jb_classify_direct_bf16": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32,
                                _c_void_p, _c_void_p, _c_void_p],
    "jb_hot_rep_bytes": [],
    "jb_df_scratch_bytes": [_i64, _i64],
    "jb_df_weigh": [_c_void_p, _i32, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64,
                    _i64, _i32, _c_void_p, _i64, _c_void_p, _c_void_p],
    "jb_serial_scratch_bytes": [_i64],
    "jb_serial_scratch_bytes_lc": [_i64, _i32],
    "jb_serial_scratch_forget": [_c_void_p],
    "jb_stepper_error": [],
    "jb_stepper_prof": [_c_void_p],
    "jb_hot_detect": [_c_void_p, _i32, _c_void_p, _i64, _i32, _i32, _i32, _c_void_p, _c_void_p,
                      _i32, _c_void_p, _c_void_p, _c_void_p],
    "jb_linear_classify": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32, _c_void_p,
                           _c_void_p],
    "jb_scale": [_c_void_p, _i64, _f32, _c_void_p],
    "jb_regression_train": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32,
                            _c_void_p, _c_void_p, _f32, _f32, _i32, _c_void_p],
    "jb_regression_estimate": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                               _c_void_p],
    "jb_signature": [_c_void_p, _c_void_p, _c_void_p, _i32, _i32, _u64, _i32, _c_void_p,
                     _c_void_p, _c_void_p],
    "jb_hamming_scan": [_c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64, _i32,
                        _i32, _i32, _c_void_p, _c_void_p],
    "jb_sparse_scan": [_c_void_p, _c_void_p, _i32, _f32, _c_void_p, _c_void_p, _c_void_p,
                       _c_void_p, _c_void_p, _i64, _i32, _c_void_p, _c_void_p],
    "jb_mix_apply": [_c_void_p, _c_void_p, _c_void_p, _i64, _f32, _c_void_p],
    "jb_classify_direct": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32, _c_void_p,
                           _c_void_p, _c_void_p],
    "jb_topk": [_i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64, _i32, _i32,
                _i32, _c_void_p, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "jb_topk_blocks": [_i64, _i32],
    "jb_topk_mq_stats": [_c_void_p],
    "jb_topk_direct_scratch": [_i32],
    "jb_topk_scratch_init": [_c_void_p, _c_void_p],
    "jb_topk_set_prof": [_c_void_p],
    "jb_topk_direct_query_path": [_c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64,
                                  _i32, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p,
                                  _c_void_p, _c_void_p, _i32, _c_void_p],
    "jb_topk_scores_direct_path": [_c_void_p, _i32, _i32, _i64, _i32, _c_void_p, _c_void_p,
                                   _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p],
    "jb_lsh_query_direct": [_c_void_p, _c_void_p, _c_void_p, _i32, _i32, _u64, _i32, _i32, _c_void_p,
                            _c_void_p, _c_void_p, _i64, _i32, _c_void_p, _c_void_p, _c_void_p,
                            _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "jb_lsh_set_rows_direct": [_c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _i32, _u64, _i32,
                               _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "jb_pool_query_direct": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32,
                             _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p,
                             _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p,
                             _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "jb_topk_scores_direct": [_c_void_p, _i32, _i32, _i64, _i32, _c_void_p, _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p],
    "jb_topk_direct_query": [_c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _i64, _i32,
                            _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                            _c_void_p, _c_void_p],
    "jb_diag_empty": [_c_void_p, _i32, _c_void_p],
    "jb_scan_train": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _i32,
                      _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                      _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _i64, _c_void_p,
                      _c_void_p],
    "jb_scan_train_profile": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                              _i32, _c_void_p, _i32, _i32, _i32, _c_void_p, _c_void_p, _c_void_p,
                              _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                              _c_void_p],
    "jb_pool_scan": [_c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _c_void_p,
                     _c_void_p, _c_void_p, _c_void_p, _i64, _c_void_p, _c_void_p, _i32, _i32,
                     _c_void_p, _c_void_p],
    "jb_pool_append": [_c_void_p, _i32, _i64, _i64, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                       _c_void_p, _c_void_p, _c_void_p],
    "jb_lof_add": [_i32, _c_void_p, _c_void_p, _i32, _i32, _i32, _i64, _c_void_p, _c_void_p,
                   _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                   _i32, _c_void_p],
    "jb_lof_mark": [_i64, _i32, _c_void_p, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                    _c_void_p],
    "jb_lof_set_lists": [_i32, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _i32, _c_void_p,
                         _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                         _c_void_p],
    "jb_lof_score": [_c_void_p, _c_void_p, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                     _c_void_p, _c_void_p, _i32, _c_void_p, _i32, _c_void_p],
    "jb_fvw_count": [_c_void_p, _i64, _c_void_p, _c_void_p, _i32, _c_void_p, _i32, _c_void_p, _i32,
                     _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "jb_fvw_emit": [_c_void_p, _i64, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p, _i32,
                    _c_void_p, _i32, _c_void_p, _u64, _c_void_p, _c_void_p, _c_void_p, _c_void_p,
                    _c_void_p, _c_void_p, _c_void_p],
    "jb_fvw_comb": [_c_void_p, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32,
                    _c_void_p, _u64, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _c_void_p],
    "jb_fvw_name_bytes": [],
    "jb_kmeanspp": [_c_void_p, _i32, _i32, _c_void_p, _c_void_p, _i32, _c_void_p, _c_void_p,
                    _c_void_p, _c_void_p, _c_void_p],
    "jb_gmm_em": [_c_void_p, _i32, _i32, _c_void_p, _c_void_p, _c_void_p, _c_void_p, _i32, _i32, _c_void_p,
                  _c_void_p],
    "jb_lloyd": [_c_void_p, _i32, _i32, _c_void_p, _c_void_p, _i32, _i32, _f32, _f32, _c_void_p,
                 _c_void_p, _c_void_p, _c_void_p],
    "jb_sqdist_mfma": [_c_void_p, _i64, _c_void_p, _i32, _i32, _c_void_p, _c_void_p, _c_void_p,
                       _c_void_p],
    "jb_argmin_rows": [_c_void_p, _i64, _i32, _c_void_p, _c_void_p],
}


def argmin_rows(D: torch.Tensor) -> torch.Tensor:
    """first minimum column of every row of D [n, k] (int32 [n]); the
    nearest-representative step of the clustering coresets"""
    _dev(D, torch.float32, "D")
    n, k = D.shape
    out = torch.empty(n, dtype=torch.int32, device=D.device)
    rc = _fn("jb_argmin_rows")(_p(D), n, k, _p(out), _stream())
    _check(rc, "jb_argmin_rows")
    return out


def sqdist(X: torch.Tensor, C: torch.Tensor) -> torch.Tensor:
    """[n, k] squared euclidean distances on the matrix cores (fp32 MFMA)."""
    _dev(X, torch.float32, "X")
    _dev(C, torch.float32, "C")
    n, d = X.shape
    k, d2 = C.shape
    if d != d2:
        raise ValueError("sqdist: dimension mismatch")
    xn2 = (X * X).sum(1).contiguous()
    cn2 = (C * C).sum(1).contiguous()
    out = torch.empty((n, k), dtype=torch.float32, device=X.device)
    rc = _fn("jb_sqdist_mfma")(_p(X), n, _p(C), k, d, _p(xn2), _p(cn2), _p(out), _stream())
    _check(rc, "jb_sqdist_mfma")
    return out


def fvw_name_bytes() -> int:
    return int(_fn("jb_fvw_name_bytes")())


_df_scratch: dict = {}


def df_weigh(row_ptr, n: int, total: int, idx, val, gw, df, diff, N0: int, L0: int, update: bool,
             sel_len=None) -> None:
    """idf / bm25 of a converted batch's global-weighted slots in place, the
    document-frequency table advanced by the batch with the sequential
    semantics when ``update`` (csrc/hip/df.hip: one launch chain)"""
    _dev(row_ptr, torch.int64, "row_ptr")
    _dev(idx, torch.int32, "idx")
    _dev(val, torch.float32, "val")
    _dev(gw, torch.uint8, "gw")
    _dev(df, torch.int64, "df")
    _dev(diff, torch.int64, "diff")
    if row_ptr.numel() < n + 1 or idx.numel() < total or val.numel() < total or gw.numel() < total \
            or diff.numel() != df.numel():
        raise ValueError("df_weigh: bad operand shapes")
    need = int(_fn("jb_df_scratch_bytes")(int(total), int(n)))
    buf = _df_scratch.get(val.device)
    if buf is None or buf.numel() < need:
        buf = torch.empty(max(need, 2 * (buf.numel() if buf is not None else 0)), dtype=torch.uint8,
                          device=val.device)
        _df_scratch[val.device] = buf
    rc = _fn("jb_df_weigh")(_p(row_ptr), n, total, _p(idx), _p(val), _p(gw), _p(df), _p(diff), int(N0), int(L0),
                            1 if update else 0, _p(buf), buf.numel(), _p(sel_len), _stream())
    _check(rc, "jb_df_weigh")


def fvw_count(buf, buf_len: int, datum_off, datum_len, n: int, srules, ns: int, nrules, nn: int,
              ncomb: int, blob, base_cnt, total_cnt, err) -> None:
    """wide converter, pass 1: base and total slots per datum (csrc/hip/fv_wide.hip)"""
    _dev(buf, torch.uint8, "buf")
    _dev(datum_off, torch.int64, "datum_off")
    _dev(datum_len, torch.int32, "datum_len")
    if datum_off.numel() < n or datum_len.numel() < n or base_cnt.numel() < n or \
            total_cnt.numel() < n or buf.numel() < buf_len:
        raise ValueError("fvw_count: bad operand shapes")
    rc = _fn("jb_fvw_count")(_p(buf), buf_len, _p(datum_off), _p(datum_len), n, _p(srules), ns,
                             _p(nrules), nn, ncomb, _p(blob), _p(base_cnt), _p(total_cnt), _p(err),
                             _stream())
    _check(rc, "jb_fvw_count")


def fvw_emit(buf, buf_len: int, datum_off, datum_len, n: int, row_ptr, srules, ns: int, nrules,
             nn: int, blob, H: int, idx, val, hs, names, gw, err) -> None:
    """wide converter, pass 2: base features into each datum's slot range"""
    total = int(row_ptr[n].item()) if n else 0
    if idx.numel() < total or val.numel() < total or hs.numel() < total or gw.numel() < total or \
            names.numel() < total * fvw_name_bytes():
        raise ValueError("fvw_emit: output shorter than the slot count")
    rc = _fn("jb_fvw_emit")(_p(buf), buf_len, _p(datum_off), _p(datum_len), n, _p(row_ptr),
                            _p(srules), ns, _p(nrules), nn, _p(blob), H, _p(idx), _p(val), _p(hs),
                            _p(names), _p(gw), _p(err), _stream())
    _check(rc, "jb_fvw_emit")


def fvw_comb(buf, n: int, row_ptr, base_cnt, srules, nrules, crules, ncomb: int, blob, H: int,
             idx, val, hs, names) -> None:
    """wide converter, pass 3: combination features of the weighted base"""
    rc = _fn("jb_fvw_comb")(_p(buf), n, _p(row_ptr), _p(base_cnt), _p(srules), _p(nrules),
                            _p(crules), ncomb, _p(blob), H, _p(idx), _p(val), _p(hs), _p(names),
                            _stream())
    _check(rc, "jb_fvw_comb")


def kmeanspp(X: torch.Tensor, w: torch.Tensor, u, m: int):
    """k-means++ seeding of m rows of X [n, d] (weights w [n]) on one
    workgroup (csrc/hip/clustering.hip), u: m host-drawn uniforms ->
    (rows list, status): status 0 ok, j + 1 when draw j found zero mass"""
    import numpy as np
    _dev(X, torch.float32, "X")
    _dev(w, torch.float32, "w")
    n, d = X.shape
    if w.numel() < n or len(u) < m or m <= 0:
        raise ValueError("kmeanspp: bad operand shapes")
    dev = X.device
    ud = torch.from_numpy(np.asarray(u[:m], dtype=np.float64)).to(dev)
    scratch = torch.empty(2 * n, dtype=torch.float32, device=dev)
    out = torch.empty(m + 1, dtype=torch.int32, device=dev)
    rc = _fn("jb_kmeanspp")(_p(X), n, d, _p(w), _p(ud), m, _p(scratch), scratch.data_ptr() + 4 * n,
                            _p(out), out.data_ptr() + 4 * m, _stream())
    _check(rc, "jb_kmeanspp")
    o = out.cpu().tolist()
    return o[:m], o[m]


def lloyd(X: torch.Tensor, w: torch.Tensor, C: torch.Tensor, iters: int, atol: float,
          rtol: float):
    """weighted Lloyd iterations on one workgroup until allclose(C', C) or
    ``iters``; C [k, d] updated in place -> (assignment [n] device int32,
    iterations run), or None when k x d does not fit the kernel's LDS"""
    _dev(X, torch.float32, "X")
    _dev(w, torch.float32, "w")
    _dev(C, torch.float32, "C")
    n, d = X.shape
    k = C.shape[0]
    if C.shape[1] != d or w.numel() < n:
        raise ValueError("lloyd: bad operand shapes")
    if 4 * (2 * k * d + k) > 64 * 1024:
        return None
    assign = torch.empty(n, dtype=torch.int32, device=X.device)
    done = torch.empty(1, dtype=torch.int32, device=X.device)
    rc = _fn("jb_lloyd")(_p(X), n, d, _p(w), _p(C), k, iters, atol, rtol, _p(assign), None,
                         _p(done), _stream())
    _check(rc, "jb_lloyd")
    return assign, int(done.item())


def gmm_em(X: torch.Tensor, w: torch.Tensor, C: torch.Tensor, var: torch.Tensor, pi: torch.Tensor,
           iters: int, assign: torch.Tensor | None = None) -> bool:
    """diagonal-covariance GMM EM on one workgroup (csrc/hip/clustering.hip
    gmm_em_kernel); C / var [k, d] and pi [k] updated in place, and (assign,
    int32 [n]) every point's most likely component. False when k x d does
    not fit the kernel's LDS (the caller keeps its own path)."""
    for t, nm in ((X, "X"), (w, "w"), (C, "C"), (var, "var"), (pi, "pi")):
        _dev(t, torch.float32, nm)
    n, d = X.shape
    k = C.shape[0]
    if C.shape[1] != d or var.shape != C.shape or pi.numel() != k or w.numel() < n:
        raise ValueError("gmm_em: bad operand shapes")
    if 4 * (4 * k * d + 2 * k) > 64 * 1024:
        return False
    if assign is not None:
        _dev(assign, torch.int32, "assign")
        if assign.numel() < n:
            raise ValueError("gmm_em: assign shorter than X")
    rc = _fn("jb_gmm_em")(_p(X), n, d, _p(w), _p(C), _p(var), _p(pi), k, iters, _p(assign), _stream())
    _check(rc, "jb_gmm_em")
    return True


def signature(row_ptr, fidx, fval, n: int, hash_num: int, seed: int, mode: int, bits, norms) -> None:
    words = (hash_num + 63) // 64
    _dev(bits, torch.int64, "bits")
    _dev(norms, torch.float32, "norms")
    if bits.numel() < n * words or norms.numel() < n or row_ptr.numel() < n + 1:
        raise ValueError("signature: bad operand shapes")
    rc = _fn("jb_signature")(_p(row_ptr), _p(fidx), _p(fval), n, hash_num, seed & (2**64 - 1),
                             mode, _p(bits), _p(norms), _stream())
    _check(rc, "jb_signature")


def hamming_scan(qbits, qnorm, nq: int, tbits, tnorm, valid, nrows: int, hash_num: int,
                 metric: int, out) -> None:
    words = (hash_num + 63) // 64
    _dev(out, torch.float32, "out")
    _dev(valid, torch.uint8, "valid")
    if (qbits.numel() < nq * words or tbits.numel() < nrows * words or out.numel() < nq * nrows
            or valid.numel() < nrows or tnorm.numel() < nrows or qnorm.numel() < nq):
        raise ValueError("hamming_scan: bad operand shapes")
    rc = _fn("jb_hamming_scan")(_p(qbits), _p(qnorm), nq, _p(tbits), _p(tnorm), _p(valid), nrows,
                                words, hash_num, metric, _p(out), _stream())
    _check(rc, "jb_hamming_scan")


TOPK_MAX_K = 128            # csrc/hip/topk.hip kTopMaxK
TOPK_MAX_WORDS = 16


def _topk_scratch(device, n: int):
    key = (str(device), "topk")
    buf = _scratch.get(key)
    if buf is None or buf[0].numel() < n:
        c = max(n, 1 << 16)
        buf = (torch.empty(c, dtype=torch.float32, device=device),
               torch.empty(c, dtype=torch.int32, device=device))
        if c >= _fn("jb_topk_direct_scratch")(1):
            # the one-launch score top-k expects its state region zeroed
            _check(_fn("jb_topk_scratch_init")(_p(buf[1]), _stream()), "jb_topk_scratch_init")
        _scratch[key] = buf
    return buf


_scratch: dict = {}


def topk_hamming(qbits, qnorm, nq: int, tbits, tnorm, valid, nrows: int, hash_num: int,
                 metric: int, k: int):
    """Fused signature scan + exact top-k (csrc/hip/topk.hip): -> (dist [nq, k],
    row [nq, k]) device tensors, +inf / INT_MAX padded."""
    words = (hash_num + 63) // 64
    if not 0 < k <= TOPK_MAX_K or words > TOPK_MAX_WORDS:
        raise ValueError("topk_hamming: k or hash_num out of range")
    _dev(valid, torch.uint8, "valid")
    _dev(tnorm, torch.float32, "tnorm")
    _dev(qnorm, torch.float32, "qnorm")
    if (qbits.numel() < nq * words or tbits.numel() < nrows * words or valid.numel() < nrows
            or tnorm.numel() < nrows or qnorm.numel() < nq):
        raise ValueError("topk_hamming: bad operand shapes")
    return _topk(0, qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num, metric, None, 0,
                 k, qbits.device)


def topk_scores(scores, nq: int, nrows: int, k: int, flip: bool):
    """Exact top-k smallest of a [nq, nrows] fp32 distance (flip: 1 - score)
    matrix -> (dist [nq, k], row [nq, k])."""
    if not 0 < k <= TOPK_MAX_K:
        raise ValueError("topk_scores: k out of range")
    _dev(scores, torch.float32, "scores")
    if scores.numel() < nq * nrows:
        raise ValueError("topk_scores: bad operand shapes")
    return _topk(1, None, None, nq, None, None, None, nrows, 0, 0, 0, scores, 1 if flip else 0, k,
                 scores.device)


def topk_mq_stats() -> list:
    """counters of the multi-query scan since the last call (JB_TOPK_MQ_STATS=1):
    survivor passes, chunks, first-chunk cuts, register pops"""
    out = (ctypes.c_ulonglong * 4)()
    _check(_fn("jb_topk_mq_stats")(ctypes.addressof(out)), "jb_topk_mq_stats")
    return list(out)


def _topk(mode, qbits, qnorm, nq, tbits, tnorm, valid, nrows, words, hash_num, metric, src, flip,
          k, device):
    blocks = _fn("jb_topk_blocks")(nrows, k)
    sd, si = _topk_scratch(device, nq * blocks * k)
    out_d = torch.empty((nq, k), dtype=torch.float32, device=device)
    out_i = torch.empty((nq, k), dtype=torch.int32, device=device)
    rc = _fn("jb_topk")(mode, _p(qbits), _p(qnorm), nq, _p(tbits), _p(tnorm), _p(valid), nrows,
                        words, hash_num, metric, _p(src), flip, k, _p(sd), _p(si), _p(out_d),
                        _p(out_i), _stream())
    _check(rc, "jb_topk")
    return out_d, out_i


def sparse_scan(qidx, qval, qnorm2: float, row_ptr, ridx, rval, rnorm2, valid, nrows: int,
                metric: int, out) -> None:
    qn = qidx.numel()
    if qn > 4096:
        raise ValueError("sparse_scan: query has more than 4096 features")
    if out.numel() < nrows or row_ptr.numel() < nrows + 1 or valid.numel() < nrows:
        raise ValueError("sparse_scan: bad operand shapes")
    rc = _fn("jb_sparse_scan")(_p(qidx), _p(qval), qn, float(qnorm2), _p(row_ptr), _p(ridx),
                               _p(rval), _p(rnorm2), _p(valid), nrows, metric, _p(out), _stream())
    _check(rc, "jb_sparse_scan")

POOL_MAX_Q = 8              # csrc/hip/sparse_pool.hip kPoolMaxQ
POOL_MAX_Q_ENTRIES = 4096   # kPoolMaxQEntries


def pool_scan(qptr, qidx, qval, qn2, nq: int, pool, nrows: int, metric: int, out,
              qslots=None, qtotal: int = 0) -> None:
    """[nq, nrows] cosine similarity (metric 0) / euclidean distance (1) of
    nq sorted sparse queries vs the rows of ``pool`` (models/similarity.py
    DevicePool), one pass over the pool. Queries are a device CSR (qptr,
    qidx, qval, qn2 [nq] float64) or, with ``qslots`` (device int32 [nq]),
    stored rows taken from the pool. ``qtotal`` = the queries' total entries
    (sizes the kernel's LDS hash table; must be exact)."""
    if not 0 < nq <= POOL_MAX_Q:
        raise ValueError("pool_scan: 1..8 queries per pass")
    _dev(out, torch.float32, "out")
    if out.numel() < nq * nrows or nrows > pool.cap_rows:
        raise ValueError("pool_scan: bad operand shapes")
    if qslots is not None:
        _dev(qslots, torch.int32, "qslots")
        if qslots.numel() < nq:
            raise ValueError("pool_scan: bad query slots")
        qptr = qidx = qval = qn2 = None
    else:
        _dev(qn2, torch.float64, "qn2")
        if qptr.numel() < nq + 1 or qidx.numel() < qtotal or qval.numel() < qtotal or \
                qn2.numel() < nq:
            raise ValueError("pool_scan: bad operand shapes")
    if not 0 <= qtotal <= POOL_MAX_Q_ENTRIES:
        raise ValueError("pool_scan: more than 4096 query entries")
    rc = _fn("jb_pool_scan")(_p(qptr), _p(qidx), _p(qval), _p(qn2), _p(qslots), nq, qtotal,
                             _p(pool.r_off), _p(pool.r_len), _p(pool.r_n2), _p(pool.valid), nrows,
                             _p(pool.p_idx), _p(pool.p_val), metric, pool.lanes_per_row(nq),
                             _p(out), _stream())
    _check(rc, "jb_pool_scan")


def pool_append(pack, n: int, nnz: int, base: int, pool) -> None:
    _dev(pack, torch.uint8, "pack")
    if pack.numel() < 32 * n + 8 * nnz or base + nnz > pool.cap_entries:
        raise ValueError("pool_append: bad operand shapes")
    rc = _fn("jb_pool_append")(_p(pack), n, nnz, base, _p(pool.r_off), _p(pool.r_len),
                               _p(pool.r_n2), _p(pool.valid), _p(pool.p_idx), _p(pool.p_val),
                               _stream())
    _check(rc, "jb_pool_append")


def _lof_check(st, *slots) -> None:
    for s in slots:
        if not 0 <= s < st.cap:
            raise ValueError("lof: slot out of range")


def lof_add(p: int, cs, cd, st, out: "HostBuffer", max_missing: int) -> None:
    """one LOF add on the device (csrc/hip/lof.hip jb_lof_add): candidates
    (host int32 / float32 arrays, the rnn nearest of p ascending, p excluded)
    in the kernel arguments, 128 per launch; insert + staleness mark + score
    of p, waited for; ``out`` = [status, score, lrd, nmissing, missing...]"""
    _lof_check(st, p)
    nc = int(cs.size)
    if cd.size < nc or cs.dtype.itemsize != 4 or cd.dtype.itemsize != 4:
        raise ValueError("lof_add: int32 / float32 candidates")
    if out.nbytes < 4 * (4 + max_missing):
        raise ValueError("lof_add: output buffer too small")
    rc = _fn("jb_lof_add")(p, cs.ctypes.data, cd.ctypes.data, nc, st.k, int(st.ignore_same),
                           st.cap, _p(st.nb_slot), _p(st.nb_dist), _p(st.kdist), _p(st.ok),
                           _p(st.lrd), _p(st.lrd_ok), _p(st._changed), _p(st._nchanged), out.ptr,
                           max_missing, _stream())
    _check(rc, "jb_lof_add")


def lof_mark(st, clear_ok: bool) -> None:
    """rows listing one of st._changed[:st._nchanged]: lrd stale (and list
    invalid when clear_ok)"""
    rc = _fn("jb_lof_mark")(st.cap, st.k, _p(st.nb_slot), _p(st._changed), _p(st._nchanged),
                            int(clear_ok), _p(st.ok), _p(st.lrd_ok), _stream())
    _check(rc, "jb_lof_mark")


def lof_set_lists(n: int, slots, cs, cd, kk: int, st) -> None:
    if slots.numel() < n or cs.numel() < n * kk or cd.numel() < n * kk:
        raise ValueError("lof_set_lists: bad operand shapes")
    rc = _fn("jb_lof_set_lists")(n, _p(slots), _p(cs), _p(cd), kk, st.k, int(st.ignore_same),
                                 _p(st.nb_slot), _p(st.nb_dist), _p(st.kdist), _p(st.ok),
                                 _p(st.lrd_ok), _p(st._changed), _p(st._nchanged), _stream())
    _check(rc, "jb_lof_set_lists")


def lof_score(ts, td, st, store: int, out: "HostBuffer", max_missing: int) -> None:
    """LOF of one point from its nearest (host int32 slots / float32
    distances, at most 64) into ``out`` = [status, score, lrd, nmissing,
    missing...]; waited for"""
    nt = int(ts.size)
    if nt > 64 or td.size < nt or ts.dtype.itemsize != 4 or td.dtype.itemsize != 4:
        raise ValueError("lof_score: at most 64 int32 / float32 targets")
    if store >= st.cap or out.nbytes < 4 * (4 + max_missing):
        raise ValueError("lof_score: bad operand shapes")
    rc = _fn("jb_lof_score")(ts.ctypes.data, td.ctypes.data, nt, st.k, _p(st.nb_slot),
                             _p(st.nb_dist), _p(st.kdist), _p(st.ok), _p(st.lrd), _p(st.lrd_ok),
                             store, out.ptr, max_missing, _stream())
    _check(rc, "jb_lof_score")


_fns: dict = {}

LABEL_CAPS = (8, 16, 32, 64, 128, 256, 512, 1024)
# storage types of the linear W table (P / S stays fp32)
W_DTYPES = (torch.float32, torch.bfloat16)
# EXACT: one stream; SERIAL: several streams with the result of applying them
# one after the other (csrc/hip/serial.hip); ATOMIC / HOGWILD: lock-free
# concurrent streams (not serial-equivalent)
UPDATE_EXACT, UPDATE_ATOMIC, UPDATE_HOGWILD, UPDATE_SERIAL = 0, 1, 2, 3
UPDATE_MODES = {"exact": UPDATE_SERIAL, "atomic": UPDATE_ATOMIC, "hogwild": UPDATE_HOGWILD}
METHODS = {"perceptron": 0, "PA": 1, "PA1": 2, "PA2": 3, "CW": 4, "AROW": 5, "NHERD": 6}


def stepper_error() -> int:
    """abort reason of a sequential-stepper launch since the last call (0:
    none; csrc/hip/stepper.hip waits time out instead of hanging)"""
    return int(_fn("jb_stepper_error")())


STEPPER_PROF_KEYS = ("step_total", "step_wait", "load_idle", "fetch_retire", "load_stuck", "meta_room",
                     "samples", "stages", "misses", "direct", "load_lookup", "fetch_issue", "load_total",
                     "meta_total", "fetch_total", "lk_iters", "lk_keys", "lk_cas", "st_read", "st_reduce",
                     "st_coef", "st_apply")


def stepper_prof() -> dict:
    """JB_STEPPER_PROF=1: shader cycles per stepper wave phase (and sample /
    stage / miss counts) since the last call"""
    import numpy as np
    out = np.zeros(32, np.uint64)
    if _fn("jb_stepper_prof")(out.ctypes.data) != 0:
        return {}
    return {k: int(v) for k, v in zip(STEPPER_PROF_KEYS, out.tolist())}


_ROCTX: list = []


def _roctx():
    """the ROCm marker library when JUBATUS_ROCTX=1 (csrc/native/jb_roctx.hpp
    is the native twin), else None"""
    if not _ROCTX:
        lib = None
        if os.environ.get("JUBATUS_ROCTX") == "1":
            for name in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1",
                         "libroctx64.so.4"):
                try:
                    lib = ctypes.CDLL(name, mode=ctypes.RTLD_GLOBAL)
                    lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                    lib.roctxRangePushA.restype = ctypes.c_int
                    lib.roctxRangePop.restype = ctypes.c_int
                    break
                except (OSError, AttributeError):
                    lib = None
        _ROCTX.append(lib)
    return _ROCTX[0]


def _fn(name: str):
    f = _fns.get(name)
    if f is None:
        lib = hip_lib()
        raw = getattr(lib, name)
        raw.argtypes = _SIGS[name]
        raw.restype = ctypes.c_int64 if name.endswith(("_bytes", "_create")) else ctypes.c_int
        tag = "hip." + name[3:]

        tx = _roctx()
        if tx is not None:
            # JUBATUS_ROCTX=1: a roctx range per kernel-group call (rocprofv3 --marker-trace)
            label = tag.encode()

            def f(*args, _raw=raw, _tag=tag, _label=label, _tx=tx):
                t0 = time.perf_counter_ns()
                _tx.roctxRangePushA(_label)
                try:
                    rc = _raw(*args)
                finally:
                    _tx.roctxRangePop()
                trace.record(_tag, time.perf_counter_ns() - t0)
                return rc
        else:
            def f(*args, _raw=raw, _tag=tag):
                t0 = time.perf_counter_ns()
                rc = _raw(*args)
                trace.record(_tag, time.perf_counter_ns() - t0)
                return rc
        _fns[name] = f
    return f


def _stream() -> int:
    return torch.cuda.current_stream().cuda_stream


def _p(t: torch.Tensor | None) -> int | None:
    return None if t is None else t.data_ptr()


def _check(rc: int, name: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{name}: HIP launch failed (code {rc})")


def _dev(t: torch.Tensor, dtype: torch.dtype, name: str) -> None:
    if not t.is_cuda or t.dtype != dtype or not t.is_contiguous():
        raise TypeError(f"{name}: expected contiguous {dtype} device tensor, got {t.dtype} "
                        f"on {t.device}")


def fv_hash(buf: torch.Tensor, buf_len: int, datum_off: torch.Tensor, datum_len: torch.Tensor,
            row_ptr: torch.Tensor, n: int, srules: torch.Tensor, n_srules: int,
            nrules: torch.Tensor, n_nrules: int, blob: torch.Tensor, H: int,
            out_idx: torch.Tensor, out_val: torch.Tensor, err: torch.Tensor) -> None:
    _dev(buf, torch.uint8, "buf")
    _dev(datum_off, torch.int64, "datum_off")
    _dev(datum_len, torch.int32, "datum_len")
    _dev(row_ptr, torch.int64, "row_ptr")
    _dev(out_idx, torch.int32, "out_idx")
    _dev(out_val, torch.float32, "out_val")
    if datum_off.numel() < n or datum_len.numel() < n or row_ptr.numel() < n + 1:
        raise ValueError("fv_hash: descriptor arrays shorter than n")
    if buf.numel() < buf_len:
        raise ValueError("fv_hash: staging buffer shorter than buf_len")
    rc = _fn("jb_fv_hash")(_p(buf), buf_len, buf.numel(), _p(datum_off), _p(datum_len),
                           _p(row_ptr), n, _p(srules), n_srules, _p(nrules), n_nrules, _p(blob),
                           blob.numel(), H, _p(out_idx), _p(out_val), _p(err), _stream())
    _check(rc, "jb_fv_hash")


def scan_train(buf: torch.Tensor, buf_used: int, req_off: torch.Tensor, req_len: torch.Tensor,
               sample_base: torch.Tensor, R: int, n: int, lt_hash: torch.Tensor,
               lt_meta: torch.Tensor, lt_blob: torch.Tensor, sps: int, spn: int,
               datum_off: torch.Tensor, datum_len: torch.Tensor, labels: torch.Tensor,
               row_ptr: torch.Tensor, req_slots: torch.Tensor, hist: torch.Tensor,
               err: torch.Tensor, empty_off: int, host_out: "HostBuffer") -> None:
    """GPU scan of R train bodies already in ``buf`` (csrc/hip/scan.hip).
    ``buf_used`` = end of the last body; the buffer needs 16 B of slack past
    it and 3 writable bytes at ``empty_off``. ``host_out`` receives [err,
    label counts...] (int32) when the batch's kernels complete."""
    for t, dt, name in ((buf, torch.uint8, "buf"), (req_off, torch.int64, "req_off"),
                        (req_len, torch.int64, "req_len"), (sample_base, torch.int64, "sample_base"),
                        (lt_hash, torch.int64, "lt_hash"), (lt_meta, torch.int32, "lt_meta"),
                        (lt_blob, torch.uint8, "lt_blob"), (datum_off, torch.int64, "datum_off"),
                        (datum_len, torch.int32, "datum_len"), (labels, torch.int32, "labels"),
                        (row_ptr, torch.int64, "row_ptr"), (req_slots, torch.int64, "req_slots"),
                        (hist, torch.int32, "hist"), (err, torch.int32, "err")):
        _dev(t, dt, name)
    cap = lt_hash.numel()
    if cap <= 0 or cap & (cap - 1) or lt_meta.numel() < 3 * cap:
        raise ValueError("scan_train: label table capacity must be a power of two")
    if req_off.numel() < R or req_len.numel() < R or sample_base.numel() < R + 1 or \
            req_slots.numel() < R:
        raise ValueError("scan_train: request arrays shorter than R")
    if datum_off.numel() < n or datum_len.numel() < n or labels.numel() < n or \
            row_ptr.numel() < n + 1:
        raise ValueError("scan_train: sample arrays shorter than n")
    if buf.numel() < buf_used + 16 or buf.numel() < empty_off + 3:
        raise ValueError("scan_train: buffer lacks the 16-B slack / the stand-in datum")
    if host_out.nbytes < 4 * (1 + hist.numel()):
        raise ValueError("scan_train: host_out shorter than 1 + len(hist) ints")
    rc = _fn("jb_scan_train")(_p(buf), _p(req_off), _p(req_len), _p(sample_base), R, _p(lt_hash),
                              _p(lt_meta), cap, _p(lt_blob), lt_blob.numel(), sps, spn,
                              _p(datum_off), _p(datum_len), _p(labels), _p(row_ptr),
                              _p(req_slots), _p(hist), hist.numel(), _p(err),
                              buf.data_ptr() + empty_off, empty_off, host_out.ptr, _stream())
    _check(rc, "jb_scan_train")


def linear_train(row_ptr: torch.Tensor, fidx: torch.Tensor, fval: torch.Tensor,
                 labels: torch.Tensor, stream_ptr: torch.Tensor, nstreams: int, W: torch.Tensor,
                 S: torch.Tensor | None, active: torch.Tensor, method: int, C: float,
                 mode: int, hot: "HotRows | None" = None, merge_every: int = 8,
                 stats: torch.Tensor | None = None, touched: torch.Tensor | None = None,
                 n_max: int = 0, scratch: "SerialScratch | None" = None) -> None:
    """mode: UPDATE_EXACT (single stream), UPDATE_SERIAL (several streams,
    serial-equivalent; needs ``scratch`` and n_max >= the batch's samples),
    UPDATE_ATOMIC or UPDATE_HOGWILD.
    hot: rows found by ``hot_detect`` for this batch (concurrent modes, label
    capacity <= 64) - kept in a block-shared LDS replica merged every
    ``merge_every`` samples. stats: int64[2] += (samples that updated,
    samples with a valid label). touched: uint8[H] rows written := 1."""
    LC = W.shape[1]
    if LC not in LABEL_CAPS:
        raise ValueError(f"label capacity {LC} not supported")
    _dev(W, W.dtype if W.dtype in W_DTYPES else torch.float32, "W")
    _dev(active, torch.int32, "active")
    if active.numel() < LC:
        raise ValueError("active mask shorter than label capacity")
    if method >= METHODS["CW"]:
        if S is None or S.shape != W.shape:
            raise ValueError("CW/AROW/NHERD need a covariance table shaped like W")
        _dev(S, torch.float32, "S")
    if stream_ptr.numel() < nstreams + 1:
        raise ValueError("stream_ptr shorter than nstreams+1")
    if stats is not None:
        _dev(stats, torch.int64, "stats")
        if stats.numel() < 2:
            raise ValueError("stats needs 2 counters")
    if touched is not None:
        _dev(touched, torch.uint8, "touched")
        if touched.numel() < W.shape[0]:
            raise ValueError("touched shorter than the table")
    if W.dtype == torch.bfloat16:
        # bf16 table: no hot-row replica; UPDATE_SERIAL runs as one
        # sequential stream (needs 16 bytes of scratch)
        if mode == UPDATE_SERIAL and scratch is None:
            raise ValueError("UPDATE_SERIAL needs scratch")
        rc = _fn("jb_linear_train_bf16")(
            _p(row_ptr), _p(fidx), _p(fval), _p(labels), _p(stream_ptr), nstreams, _p(W),
            _p(S) if S is not None else None, _p(active), LC, method, float(C), int(mode),
            _p(stats), _p(touched), scratch.ptr(max(n_max, 1), LC) if scratch is not None else None,
            scratch.nbytes if scratch is not None else 0, _stream())
        _check(rc, "jb_linear_train_bf16")
        return
    rc = _fn("jb_linear_train")(_p(row_ptr), _p(fidx), _p(fval), _p(labels), _p(stream_ptr),
                                nstreams, _p(W), _p(S) if S is not None else None, _p(active), LC,
                                method, float(C), int(mode),
                                _p(hot.rows) if hot is not None else None,
                                _p(hot.n) if hot is not None else None,
                                _p(hot.rep) if hot is not None else None, int(merge_every),
                                HOT_WAVES,
                                _p(stats), _p(touched), int(n_max),
                                scratch.ptr(n_max, LC) if scratch is not None else None,
                                scratch.nbytes if scratch is not None else 0, _stream())
    _check(rc, "jb_linear_train")


class SerialScratch:
    """device scratch of the serial-equivalent train mode (csrc/hip/serial.hip:
    the committer's tail range and the per-sample slack), grown on demand.
    Growth synchronises the device (the old buffer may still be in use)."""

    def __init__(self, device):
        self.device = device
        self.buf = None
        self.nbytes = 0

    def last_batch(self) -> dict:
        """diagnostics of the last kSerial batch (synchronises): first sample
        left to the sequential kernel, batch end, exact steps, rounds"""
        if self.buf is None:
            return {}
        v = self.buf[:256].view(torch.int64).tolist()
        reasons = ("done", "saturated", "dense", "rescore")
        out = {"tail_start": v[0], "end": v[1], "exact_steps": v[2], "rounds": v[3],
               "segments": v[21], "stop_reason": reasons[v[20]] if 0 <= v[20] < 4 else v[20]}
        if v[31] == 1:
            # verified committer (csrc/hip/vcommit.hip): windows, verification
            # retries, candidates the committer walked, non-candidates cleared
            # by the bound, the window length / threshold T it ends with
            import struct
            out.update(verified=True, windows=v[21] - v[28], retries=v[28], saturated_windows=v[29],
                       candidates=v[27], non_candidates_verified=v[7], committer_updates=v[24],
                       wasted_steps=v[22], refreshes=v[23], exact_rescored=v[26], last_segment_rows=v[25],
                       window_len=v[8], T=round(struct.unpack("f", struct.pack("I", v[9] & 0xffffffff))[0], 4),
                       commit_kernel_us=round(v[30] / 100.0, 1),
                       # samples the sequential stepper (csrc/hip/stepper.hip)
                       # applied: chunks after update-dense windows, and the
                       # rest the segments left (stop_reason "dense")
                       stepper_samples=v[16] + v[1] - v[0], stepper_chunks=v[17],
                       # windows whose candidates the stepper walked (kernel C's place)
                       stepper_windows=v[19])
            if v[15] > 0:      # JB_COMMIT_PROF=1: committer phases (shader cycles -> us by the wall clock)
                us = (v[30] / 100.0) / v[15]
                for i, nm in enumerate(("round_start", "select", "decide", "apply", "correct")):
                    out[f"commit_{nm}_us"] = round(v[10 + i] * us, 1)
            return out
        if v[24] > 0 or v[22] > 0:
            # delta committer (csrc/hip/commit.hip): steps that did not update,
            # guard-band re-scores, updates, rows in the LDS store at the end
            out.update(wasted_steps=v[22], refreshes=v[23], committer_updates=v[24],
                       last_segment_rows=v[25])
            if v[27] > 0:     # counted with the phase stamps only (JB_COMMIT_PROF=1)
                out.update(exact_rescored=v[26], committed_samples=v[27])
        # committer phases in shader cycles, scaled to us by the wall clock
        wall_us = v[10] / 100.0
        if v[11] > 0:
            us = wall_us / v[11]
            out["commit_us"] = round(wall_us, 1)
            names = (("start", "barrier_a", "step", "corr", "flush", "init") if "committer_updates" in out
                     else ("bound", "barrier_a", "stage_b1", "step", "barrier_b2", "round"))
            for i, nm in enumerate(names):
                out[f"commit_{nm}_us"] = round(v[4 + i] * us, 1)
            for w in range(8):     # per wave: round-start bounds + post-step work
                out[f"commit_wave{w}_work_us"] = round(v[12 + w] * us, 1)
        return out

    def ptr(self, n_max: int, lc: int = 0) -> int:
        """lc: the model's label capacity (0: the largest need, any capacity)"""
        need = int(_fn("jb_serial_scratch_bytes_lc")(int(n_max), int(lc)) if lc > 0
                   else _fn("jb_serial_scratch_bytes")(int(n_max)))
        if need > self.nbytes:
            if self.buf is not None:
                torch.cuda.synchronize(self.device)
            self.nbytes = max(need, 2 * self.nbytes)
            self.buf = torch.empty(self.nbytes, dtype=torch.uint8, device=self.device)
            # a new buffer starts without the segment history of whatever
            # buffer had its address before (csrc/hip/serial.hip)
            _fn("jb_serial_scratch_forget")(self.buf.data_ptr())
        return self.buf.data_ptr()


HOT_MAX_ROWS = 64           # csrc/hip/linear.hip Hot<LC>::R (LC = 8)
# streams (waves) per block of a hot launch: 4, 8 or 16 (JUBATUS_HOT_WAVES)
HOT_WAVES = int(__import__("os").environ.get("JUBATUS_HOT_WAVES", "8"))
HOT_ENTRIES = 512           # Hot<LC>::E: hot rows x label capacity


def hot_max_rows(LC: int) -> int:
    return min(HOT_MAX_ROWS, HOT_ENTRIES // LC)


class HotRows:
    """device hot-row list of one batch, the candidate table hot_detect
    leaves empty after every call (csrc/hip/hot.hip) and the train kernel's
    delta shards (csrc/hip/linear.hip "Hot rows"; left zero by every launch)"""

    CAP = 1 << 14

    def __init__(self, device):
        self.rows = torch.zeros(HOT_MAX_ROWS, dtype=torch.int32, device=device)
        self.n = torch.zeros(1, dtype=torch.int32, device=device)
        self.rep = torch.zeros(_fn("jb_hot_rep_bytes")() // 4, dtype=torch.float32, device=device)
        self.free = DevEvent()  # recorded after the train launch that read this set
        self.free_used = False  # recorded at least once
        self.gkey = torch.full((self.CAP,), -1, dtype=torch.int32, device=device)
        self.gcnt = torch.zeros(self.CAP, dtype=torch.int32, device=device)


def hot_detect(row_ptr: torch.Tensor, n: int, fidx: torch.Tensor, max_slots: int, hot: HotRows,
               min_count: int, block_min: int = 8, max_rows: int = HOT_MAX_ROWS) -> None:
    """rows carried by at least ``min_count`` of the batch's feature slots
    -> hot.rows[:hot.n] (device; no host synchronisation)"""
    _dev(row_ptr, torch.int64, "row_ptr")
    _dev(fidx, torch.int32, "fidx")
    if row_ptr.numel() < n + 1 or fidx.numel() < max_slots:
        raise ValueError("hot_detect: bad operand shapes")
    max_rows = min(max_rows, hot.rows.numel())
    rc = _fn("jb_hot_detect")(_p(row_ptr), n, _p(fidx), int(max_slots), int(block_min),
                              int(min_count), int(max_rows), _p(hot.gkey), _p(hot.gcnt),
                              hot.CAP, _p(hot.rows), _p(hot.n), _stream())
    _check(rc, "jb_hot_detect")


def linear_classify(row_ptr: torch.Tensor, fidx: torch.Tensor, fval: torch.Tensor, n: int,
                    W: torch.Tensor, out: torch.Tensor) -> None:
    LC = W.shape[1]
    if LC not in LABEL_CAPS:
        raise ValueError(f"label capacity {LC} not supported")
    _dev(W, W.dtype if W.dtype in W_DTYPES else torch.float32, "W")
    _dev(out, torch.float32, "out")
    if out.numel() < n * LC or row_ptr.numel() < n + 1:
        raise ValueError("linear_classify: output / row_ptr too small")
    fn = "jb_linear_classify_bf16" if W.dtype == torch.bfloat16 else "jb_linear_classify"
    rc = _fn(fn)(_p(row_ptr), _p(fidx), _p(fval), n, _p(W), LC, _p(out), _stream())
    _check(rc, fn)


def mix_apply_(w: torch.Tensor, red: torch.Tensor, loc: torch.Tensor, inv_n: float) -> None:
    """w += red * inv_n - loc (overlapped MIX finish)"""
    for name, t in (("w", w), ("red", red), ("loc", loc)):
        _dev(t, torch.float32, name)
    if not (w.numel() == red.numel() == loc.numel()):
        raise ValueError("mix_apply_: size mismatch")
    rc = _fn("jb_mix_apply")(_p(w), _p(red), _p(loc), w.numel(), float(inv_n), _stream())
    _check(rc, "jb_mix_apply")


def scale_(t: torch.Tensor, a: float) -> None:
    _dev(t, torch.float32, "t")
    rc = _fn("jb_scale")(_p(t), t.numel(), float(a), _stream())
    _check(rc, "jb_scale")


def regression_train(row_ptr, fidx, fval, targets, stream_ptr, nstreams: int, W, stats,
                     C: float, eps: float, concurrent: bool) -> None:
    _dev(W, torch.float32, "W")
    _dev(stats, torch.float32, "stats")
    _dev(targets, torch.float32, "targets")
    if W.dim() != 1 or stats.numel() < 3 or stream_ptr.numel() < nstreams + 1:
        raise ValueError("regression_train: bad operand shapes")
    rc = _fn("jb_regression_train")(_p(row_ptr), _p(fidx), _p(fval), _p(targets), _p(stream_ptr),
                                    nstreams, _p(W), _p(stats), float(C), float(eps),
                                    1 if concurrent else 0, _stream())
    _check(rc, "jb_regression_train")


def regression_estimate(row_ptr, fidx, fval, n: int, W, out) -> None:
    _dev(W, torch.float32, "W")
    _dev(out, torch.float32, "out")
    if out.numel() < n or row_ptr.numel() < n + 1:
        raise ValueError("regression_estimate: bad operand shapes")
    rc = _fn("jb_regression_estimate")(_p(row_ptr), _p(fidx), _p(fval), n, _p(W), _p(out),
                                       _stream())
    _check(rc, "jb_regression_estimate")


# ------------------------------------------------------- train batch submit
class DevEvent:
    """A HIP event owned by the caller (csrc/hip/train_batch.hip event API):
    the events of the one-call train batch submit. Duck-types the parts of
    torch.cuda.Event the pipeline uses (query / synchronize / record)."""

    def __init__(self):
        self.h = int(_fn("jb_event_create")())
        if not self.h:
            raise RuntimeError("hipEventCreate failed")
        self._destroy = _fn("jb_event_destroy")

    def record(self, stream: int | None = None) -> None:
        _check(_fn("jb_event_record")(self.h, _stream() if stream is None else stream),
               "jb_event_record")

    def wait_on(self, stream: int | None = None) -> None:
        """make ``stream`` (default: the current one) wait for this event"""
        _check(_fn("jb_stream_wait_event")(_stream() if stream is None else stream, self.h),
               "jb_stream_wait_event")

    def query(self) -> bool:
        rc = _fn("jb_event_query")(self.h)
        if rc not in (0, 1):
            raise RuntimeError(f"hipEventQuery failed (code {rc})")
        return rc == 0

    def synchronize(self) -> None:
        _check(_fn("jb_event_sync")(self.h), "jb_event_sync")

    def __del__(self):
        if getattr(self, "h", 0):
            self._destroy(self.h)
            self.h = 0


def stream_wait(ev, stream=None) -> None:
    """make ``stream`` (a torch stream; default the current one) wait for a
    torch.cuda.Event or a DevEvent"""
    if isinstance(ev, DevEvent):
        ev.wait_on(None if stream is None else stream.cuda_stream)
    elif stream is None:
        torch.cuda.current_stream().wait_event(ev)
    else:
        stream.wait_event(ev)


_TB_FIELDS = """copy_stream prep_stream compute_stream copy_done check_done ready set_free hot_free
hot_seen arena used:i meta_host R:i n:i d_buf buf_cap:i empty_off:i d_meta d_off d_len d_lab d_row
d_slots d_hist nhist:i d_err host_out lt_hash lt_meta lt_cap:i lt_blob lt_blob_len:i sps:i spn:i
srules nrules n_srules:i n_nrules:i blob blob_len:i H:i d_idx d_val slot_cap:i hash_err hot_rows
hot_n hot_rep gkey gcnt gcap:i block_min:i min_count:i max_rows:i hot_free_valid:i hot_count_host
W S active LC:i method:i C:d mode:i merge_every:i hot_waves:i stats touched serial_scratch
serial_bytes:i w_bf16:i""".split()


class TrainBatchArgs(ctypes.Structure):
    """csrc/hip/train_batch.hip JbTrainBatch (every field 8 bytes; the
    unsuffixed names are pointers / handles)"""
    _fields_ = [(f.split(":")[0], {"i": _i64, "d": ctypes.c_double}.get(f.partition(":")[2],
                                                                        _c_void_p))
                for f in _TB_FIELDS]


def train_batch_submit(a: TrainBatchArgs) -> None:
    """one call: H2D -> scan -> fv_hash -> [hot detect] -> train (see
    csrc/hip/train_batch.hip); the caller has checked the capacities"""
    global _tb_checked
    if not _tb_checked:
        want = int(_fn("jb_train_batch_args_bytes")())
        if want != ctypes.sizeof(TrainBatchArgs):
            raise RuntimeError(f"TrainBatchArgs is {ctypes.sizeof(TrainBatchArgs)} bytes, "
                               f"the library expects {want}")
        _tb_checked = True
    _check(_fn("jb_train_batch_submit")(ctypes.addressof(a)), "jb_train_batch_submit")


_tb_checked = False


# ------------------------------------------------------------ direct classify
DIRECT_MAX_SAMPLES = 32     # csrc/hip/classify_direct.hip kDirectMaxSamples
DIRECT_MAX_SLOTS = 320      # kDirectMaxSlots


class HostBuffer:
    """Fine-grained pinned host memory (hipHostMallocCoherent) that kernels
    write into directly; exposed to the host as a numpy array."""

    def __init__(self, nbytes: int):
        lib = hip_lib()
        lib.jb_host_alloc.restype = ctypes.c_void_p
        lib.jb_host_alloc.argtypes = [_i64]
        lib.jb_host_free.argtypes = [_c_void_p]
        self._lib = lib
        self.nbytes = int(nbytes)
        self.ptr = lib.jb_host_alloc(self.nbytes)
        if not self.ptr:
            raise MemoryError(f"hipHostMalloc({nbytes}) failed")
        ctypes.memset(self.ptr, 0, self.nbytes)

    def view(self, dtype, count: int, offset: int = 0):
        import numpy as np
        dt = np.dtype(dtype)
        if offset + count * dt.itemsize > self.nbytes:
            raise ValueError("HostBuffer view out of range")
        buf = (ctypes.c_uint8 * (count * dt.itemsize)).from_address(self.ptr + offset)
        return np.frombuffer(buf, dtype=dt, count=count)

    def __del__(self):
        if getattr(self, "ptr", None):
            self._lib.jb_host_free(self.ptr)
            self.ptr = None


def classify_direct(idx_ptr: int, val_ptr: int, row_ptr_ptr: int, n: int, W: torch.Tensor,
                    out: HostBuffer, done: HostBuffer, stream: int | None = None) -> bool:
    """Scores of n host-hashed datums (host CSR pointers) computed by ONE
    launch whose kernel arguments carry the (idx, val) pairs; the scores land
    in ``out`` (n x LC fp32). Returns False when the request does not fit the
    direct path (the caller uses the batch path)."""
    LC = W.shape[1]
    if LC not in LABEL_CAPS:
        raise ValueError(f"label capacity {LC} not supported")
    _dev(W, W.dtype if W.dtype in W_DTYPES else torch.float32, "W")
    if out.nbytes < n * LC * 4 or done.nbytes < 4 * n:
        raise ValueError("classify_direct: output buffer too small")
    fn = "jb_classify_direct_bf16" if W.dtype == torch.bfloat16 else "jb_classify_direct"
    rc = _fn(fn)(idx_ptr, val_ptr, row_ptr_ptr, n, _p(W), LC, out.ptr, done.ptr,
                 _stream() if stream is None else stream)
    if rc == 1:
        return False
    _check(rc, fn)
    return True


def diag_empty(done: HostBuffer, spin: bool, stream: int | None = None) -> None:
    rc = _fn("jb_diag_empty")(done.ptr, 1 if spin else 0, _stream() if stream is None else stream)
    _check(rc, "jb_diag_empty")


QUERY_MAX = 8          # csrc/hip/lsh.hip kQueryMax


def _direct_scratch(nrows: int, k: int, nq: int) -> int:
    """scratch of the latency top-k: tile path (blocks * k) or sampled path"""
    return max(nq * _fn("jb_topk_blocks")(nrows, k) * k, _fn("jb_topk_direct_scratch")(nq))
QUERY_SLOTS = 256      # kQuerySlots


class DirectQueryBuffers:
    """pinned host outputs + device scratch of the LSH latency path"""

    def __init__(self, device, words: int):
        self.out_d = HostBuffer(QUERY_MAX * TOPK_MAX_K * 4)
        self.out_i = HostBuffer(QUERY_MAX * TOPK_MAX_K * 4)
        self.done = HostBuffer(QUERY_MAX * 4)
        self.qbits = torch.empty(QUERY_MAX * max(words, 1), dtype=torch.int64, device=device)
        self.qnorm = torch.empty(QUERY_MAX, dtype=torch.float32, device=device)


def lsh_query_direct(idx_ptr: int, val_ptr: int, row_ptr_ptr: int, nq: int, hash_num: int, seed: int,
                     mode: int, metric: int, tbits, tnorm, valid, nrows: int, k: int,
                     bufs: DirectQueryBuffers, stream: int | None = None):
    """-> (dist [nq, k], row [nq, k]) numpy (copies), or None when the query
    does not fit the direct path"""
    import numpy as np
    words = (hash_num + 63) // 64
    if not (0 < k <= TOPK_MAX_K and words <= TOPK_MAX_WORDS and 0 < nq <= QUERY_MAX):
        return None
    _dev(valid, torch.uint8, "valid")
    _dev(tnorm, torch.float32, "tnorm")
    if tbits.numel() < nrows * words or valid.numel() < nrows or tnorm.numel() < nrows:
        raise ValueError("lsh_query_direct: bad table shapes")
    sd, si = _topk_scratch(tbits.device, _direct_scratch(nrows, k, nq))
    rc = _fn("jb_lsh_query_direct")(idx_ptr, val_ptr, row_ptr_ptr, nq, hash_num, seed & (2**64 - 1),
                                    mode, metric, _p(tbits), _p(tnorm), _p(valid), nrows, k,
                                    _p(bufs.qbits), _p(bufs.qnorm), _p(sd), _p(si), bufs.out_d.ptr,
                                    bufs.out_i.ptr, bufs.done.ptr,
                                    _stream() if stream is None else stream)
    if rc == 1:
        return None
    _check(rc, "jb_lsh_query_direct")
    d = bufs.out_d.view(np.float32, nq * k).reshape(nq, k).copy()
    i = bufs.out_i.view(np.int32, nq * k).reshape(nq, k).copy()
    return d, i


def topk_scores_direct(scores, nq: int, nrows: int, k: int, flip: bool,
                       bufs: DirectQueryBuffers, path: int = -1):
    """exact top-k smallest of a [nq, nrows] score matrix (flip: 1 - score)
    -> (dist [nq, k], row [nq, k]) numpy; sampled threshold + collect + final
    merge written to pinned host memory and waited for (csrc/hip/topk.hip
    jb_topk_scores_direct; path >= 0 forces a path: 0 tile, 1 radix chain,
    2 one launch with grid barriers, 3 one pass, k <= 16)"""
    import numpy as np
    if not (0 < k <= TOPK_MAX_K and 0 < nq <= QUERY_MAX):
        raise ValueError("topk_scores_direct: k / nq out of range")
    _dev(scores, torch.float32, "scores")
    if scores.numel() < nq * nrows:
        raise ValueError("topk_scores_direct: bad operand shapes")
    sd, si = _topk_scratch(scores.device, _direct_scratch(nrows, k, nq))
    rc = _fn("jb_topk_scores_direct_path")(_p(scores), 1 if flip else 0, nq, nrows, k, _p(sd), _p(si),
                                           bufs.out_d.ptr, bufs.out_i.ptr, bufs.done.ptr, path, _stream())
    _check(rc, "jb_topk_scores_direct")
    d = bufs.out_d.view(np.float32, nq * k).reshape(nq, k).copy()
    i = bufs.out_i.view(np.int32, nq * k).reshape(nq, k).copy()
    return d, i


def pool_query_direct(pool, nrows: int, metric: int, k: int, bufs: DirectQueryBuffers,
                      idx=None, val=None, row_ptr=None, slots=None, nq: int = 0):
    """latency path of the device inverted index (csrc/hip/sparse_pool.hip
    jb_pool_query_direct): nq host queries - a hashed CSR (numpy int32 /
    float32 / int64; normalized natively) or stored-row slots - scored with
    the query in the kernel arguments, exact top-k returned from pinned
    memory -> (dist [nq, k], row [nq, k]) numpy, or None when the query does
    not fit the kernel arguments. Distances: euclidean, or 1 - cosine."""
    import numpy as np
    if not (0 < k <= TOPK_MAX_K and 0 < nq <= POOL_MAX_Q) or nrows <= 0:
        return None
    if nrows > pool.cap_rows:
        raise ValueError("pool_query_direct: nrows beyond the pool")
    sd, si = _topk_scratch(pool.device, _direct_scratch(nrows, k, nq))
    scores = pool.score_scratch(nq * nrows)
    if slots is not None:
        slots = np.ascontiguousarray(slots, dtype=np.int32)
        if slots.size < nq or int(slots.max()) >= pool.cap_rows or int(slots.min()) < 0:
            raise ValueError("pool_query_direct: bad slots")
        slen = np.ascontiguousarray(pool.len_h[slots], dtype=np.int64)
        args = (None, None, None, slots.ctypes.data, slen.ctypes.data)
    else:
        if row_ptr.dtype != np.int64 or idx.dtype != np.int32 or val.dtype != np.float32 or \
                row_ptr.size < nq + 1 or idx.size < row_ptr[nq] or val.size < row_ptr[nq]:
            raise ValueError("pool_query_direct: bad query CSR")
        args = (idx.ctypes.data, val.ctypes.data, row_ptr.ctypes.data, None, None)
    rc = _fn("jb_pool_query_direct")(*args, nq, _p(pool.r_off), _p(pool.r_len), _p(pool.r_n2),
                                     _p(pool.valid), nrows, _p(pool.p_idx), _p(pool.p_val),
                                     metric, pool.lanes_per_row(nq), k, _p(scores), _p(sd), _p(si),
                                     bufs.out_d.ptr, bufs.out_i.ptr, bufs.done.ptr, _stream())
    if rc == 1:
        return None
    _check(rc, "jb_pool_query_direct")
    d = bufs.out_d.view(np.float32, nq * k).reshape(nq, k).copy()
    i = bufs.out_i.view(np.int32, nq * k).reshape(nq, k).copy()
    return d, i


def lsh_set_rows_direct(idx_ptr: int, val_ptr: int, row_ptr_ptr: int, n: int, slots_ptr: int,
                        hash_num: int, seed: int, mode: int, tbits, tnorm, valid) -> bool:
    """signatures of n host-hashed rows written into their table slots by one
    launch whose arguments carry the rows (async). False: does not fit."""
    _dev(valid, torch.uint8, "valid")
    _dev(tnorm, torch.float32, "tnorm")
    rc = _fn("jb_lsh_set_rows_direct")(idx_ptr, val_ptr, row_ptr_ptr, n, slots_ptr, hash_num,
                                       seed & (2**64 - 1), mode, _p(tbits), _p(tnorm), _p(valid),
                                       _stream())
    if rc == 1:
        return False
    _check(rc, "jb_lsh_set_rows_direct")
    return True


def topk_rows_direct(qbits, qnorm, nq: int, tbits, tnorm, valid, nrows: int, hash_num: int,
                     metric: int, k: int, bufs: DirectQueryBuffers, path: int = -1):
    """queries whose signatures are device rows (gathered table rows): fused
    scan/top-k straight into pinned host memory -> numpy (dist, row) or None
    (path >= 0 forces a path: 0 tile, 2 one launch with grid barriers, 3 one
    pass, k <= 16)"""
    import numpy as np
    words = (hash_num + 63) // 64
    if not (0 < k <= TOPK_MAX_K and words <= TOPK_MAX_WORDS and 0 < nq <= QUERY_MAX):
        return None
    sd, si = _topk_scratch(tbits.device, _direct_scratch(nrows, k, nq))
    rc = _fn("jb_topk_direct_query_path")(_p(qbits), _p(qnorm), nq, _p(tbits), _p(tnorm), _p(valid),
                                         nrows, words, hash_num, metric, k, _p(sd), _p(si),
                                         bufs.out_d.ptr, bufs.out_i.ptr, bufs.done.ptr, path, _stream())
    _check(rc, "jb_topk_direct_query")
    d = bufs.out_d.view(np.float32, nq * k).reshape(nq, k).copy()
    i = bufs.out_i.view(np.int32, nq * k).reshape(nq, k).copy()
    return d, i
