"""Pure-NumPy reference of the online linear classifiers.

This is the numerical oracle for csrc/hip/linear.hip and the CPU backend of
the classifier engine. One call of ``train_one`` applies exactly one online
update; a sequence of calls is the exact sequential semantics of one
``train`` request (reference: jubatus/server/server/classifier_serv.cpp:138-144).

Notation for one sample (x, y): s_l = sum_i x_i W[i,l]; l* = best-scoring
active label other than y (lowest index on ties; none if y is the only
label); margin m = s_y - s_l* (s_l* := 0 without l*); ||x||^2 = sum_i x_i^2;
v = sum_i x_i^2 (S[i,y] + S[i,l*]).

  perceptron  m <= 0:  W_y += x, W_l* -= x
  PA          loss = 1 - m > 0: tau = loss / (k ||x||^2), k = 2 (1 without l*)
  PA1         tau = min(C, loss / (k ||x||^2))
  PA2         tau = loss / (k ||x||^2 + 1/(2C))
              W_y += tau x, W_l* -= tau x
  CW          phi = C, b = 1 + 2 phi m,
              gamma = (-b + sqrt(b^2 - 8 phi (m - phi v))) / (4 phi v) > 0:
              W_y += gamma S_y x, W_l* -= gamma S_l* x,
              S <- 1 / (1/S + 2 gamma phi x^2)            (both labels)
  AROW        m < 1: beta = 1 / (v + 1/C), alpha = (1 - m) beta
              W_y += alpha S_y x, W_l* -= alpha S_l* x, S -= beta S^2 x^2
  NHERD       m < 1: alpha = (1 - m) / (v + 1/C)
              W as AROW; S -= S^2 x^2 (C^2 v + 2C) / (1 + C v)^2

The diagonal covariance S is *stored as its precision* P = 1/S (init 1):
the updates above become additive, P += beta x^2 (CW) and
P += beta x^2 / (1 - beta S x^2) (AROW, NHERD) - algebraically identical,
always positive, and commutative (what lets concurrent GPU streams apply
them with float atomics).

Coordinates with idx < 0 are ignored. Every update reads the table before
the sample and then adds its increments (gather-compute-scatter), like the
kernel; a row that occurs twice in one sample receives both increments
(the reference's per-feature update loop does the same).
"""
from __future__ import annotations

import math

import numpy as np

PERCEPTRON, PA, PA1, PA2, CW, AROW, NHERD = range(7)
METHOD_IDS = {"perceptron": PERCEPTRON, "PA": PA, "PA1": PA1, "PA2": PA2, "CW": CW,
              "AROW": AROW, "NHERD": NHERD}
USES_COVARIANCE = {CW, AROW, NHERD}


def scores(W: np.ndarray, idx: np.ndarray, val: np.ndarray) -> np.ndarray:
    m = idx >= 0
    return (val[m, None].astype(np.float32) * W[idx[m]]).sum(axis=0, dtype=np.float32)


def train_one(W: np.ndarray, P: np.ndarray | None, idx: np.ndarray, val: np.ndarray, y: int,
              active: np.ndarray, method: int, C: float) -> bool:
    m = idx >= 0
    idx = idx[m]
    x = val[m].astype(np.float32)
    s = (x[:, None] * W[idx]).sum(axis=0, dtype=np.float32) if len(idx) else \
        np.zeros(W.shape[1], np.float32)
    sy = float(s[y])
    best, lstar = -math.inf, -1
    for l in range(W.shape[1]):
        if active[l] and l != y and s[l] > best:
            best, lstar = float(s[l]), l
    margin = sy - (best if lstar >= 0 else 0.0)
    nrm = float((x * x).sum())
    use_s = method in USES_COVARIANCE
    if use_s:
        a = (np.float32(1.0) / P[idx, y]).astype(np.float32)
        b = ((np.float32(1.0) / P[idx, lstar]).astype(np.float32) if lstar >= 0
             else np.zeros_like(a))
        var = float((x * x * (a + b)).sum())
    else:
        a = b = None
        var = 0.0
    tau = beta = 0.0
    if method == PERCEPTRON:
        if margin > 0:
            return False
        tau = 1.0
    elif method in (PA, PA1, PA2):
        loss = 1.0 - margin
        if loss <= 0 or nrm <= 0:
            return False
        sq = (2.0 if lstar >= 0 else 1.0) * nrm
        tau = loss / sq if method == PA else (min(C, loss / sq) if method == PA1
                                              else loss / (sq + 0.5 / C))
    elif method == CW:
        if var <= 0:
            return False
        phi = C
        bb = 1.0 + 2.0 * phi * margin
        disc = bb * bb - 8.0 * phi * (margin - phi * var)
        gamma = (-bb + math.sqrt(max(disc, 0.0))) / (4.0 * phi * var)
        if gamma <= 0:
            return False
        tau, beta = gamma, 2.0 * gamma * phi
    elif method == AROW:
        if margin >= 1.0:
            return False
        beta = 1.0 / (var + 1.0 / C)
        tau = (1.0 - margin) * beta
    elif method == NHERD:
        if margin >= 1.0:
            return False
        tau = (1.0 - margin) / (var + 1.0 / C)
        cv = 1.0 + C * var
        beta = (C * C * var + 2.0 * C) / (cv * cv)
    else:
        raise ValueError(f"unknown method {method}")
    if use_s:
        np.add.at(W, (idx, y), (np.float32(tau) * a * x).astype(np.float32))
        if lstar >= 0:
            np.add.at(W, (idx, lstar), (-np.float32(tau) * b * x).astype(np.float32))
        bx2 = np.float32(beta) * x * x
        if method == CW:
            dy = dl = bx2
        else:
            dy = bx2 / (np.float32(1.0) - bx2 * a)
            dl = bx2 / (np.float32(1.0) - bx2 * b)
        np.add.at(P, (idx, y), dy.astype(np.float32))
        if lstar >= 0:
            np.add.at(P, (idx, lstar), dl.astype(np.float32))
    else:
        np.add.at(W, (idx, y), (np.float32(tau) * x).astype(np.float32))
        if lstar >= 0:
            np.add.at(W, (idx, lstar), (-np.float32(tau) * x).astype(np.float32))
    return True
