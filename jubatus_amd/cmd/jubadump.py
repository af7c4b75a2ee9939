"""jubadump: model file -> JSON (the reference's separate jubadump package,
man/en/jubadump.1). Reads a model file written by ``save`` (CRC-checked
container, framework/save_load.py; nothing in it is executed) and prints the
system data plus the engine payload as JSON. Linear-classifier payloads are
expanded to per-row weights: {"weights": {"<row>": {"<label>": w}}} (rows are
feature-hash slots - feature names are not stored in the model, exactly as
with a hashed reference model); other binary blobs print as their sizes.

Usage: python -m jubatus_amd.cmd.jubadump -i MODEL_FILE
"""
from __future__ import annotations

import argparse
import base64
import json
import sys

import numpy as np

from ..framework.save_load import ModelFileError, read_model_file


def _plain(x):
    if isinstance(x, bytes):
        try:
            return x.decode()
        except UnicodeDecodeError:
            return {"binary_bytes": len(x), "base64_head": base64.b64encode(x[:48]).decode()}
    if isinstance(x, dict):
        return {str(_plain(k)): _plain(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return [_plain(v) for v in x]
    return x


def expand_linear(p: dict) -> dict:
    labels = [_plain(x) for x in p["labels"]]
    rows = np.frombuffer(p["rows"], dtype=np.int64)
    L = len(labels)
    W = np.frombuffer(p["W"], dtype=np.float32).reshape(len(rows), L) if L else np.zeros((len(rows), 0))
    out = {"method": _plain(p["method"]), "hash_max_size": int(p["H"]),
           "labels": dict(zip(labels, [int(c) for c in p["counts"]])),
           "weights": {str(int(r)): {lab: float(W[i, j]) for j, lab in enumerate(labels) if W[i, j] != 0.0}
                       for i, r in enumerate(rows)}}
    if len(p.get("P") or b""):
        P = np.frombuffer(p["P"], dtype=np.float32).reshape(len(rows), L)
        out["covariance"] = {str(int(r)): {lab: float(1.0 / P[i, j]) for j, lab in enumerate(labels)
                                           if P[i, j] != 1.0} for i, r in enumerate(rows)}
    return out


def dump(path: str) -> dict:
    with open(path, "rb") as f:
        sysobj, userobj = read_model_file(f)
    version, ts, typ, mid, config = [_plain(x) for x in sysobj]
    payload = userobj[1]
    if isinstance(payload, dict):
        p = {(k.decode() if isinstance(k, bytes) else k): v for k, v in payload.items()}
        body = expand_linear(p) if {"rows", "W", "labels", "H"} <= set(p) else _plain(p)
    else:
        body = _plain(payload)
    try:
        config = json.loads(config)
    except (TypeError, json.JSONDecodeError):
        pass
    return {"system": {"version": version, "timestamp": ts, "type": typ, "id": mid,
                       "config": config, "user_data_version": userobj[0]},
            "model": body}


def main(argv: list[str] | None = None, out=None) -> int:
    out = out or sys.stdout
    p = argparse.ArgumentParser(prog="jubadump")
    p.add_argument("-i", "--input", required=True)
    a = p.parse_args(argv)
    try:
        out.write(json.dumps(dump(a.input), indent=1, sort_keys=True) + "\n")
    except (OSError, ModelFileError) as e:
        sys.stderr.write(f"jubadump: {e}\n")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
