"""Device conversion for the wide rule set (csrc/hip/fv_wide.hip): ngram /
space splitters, tf / log_tf sample weights, idf / bm25 global weights
against a document-frequency table in HBM, num / log rules and add / mul
combinations. Equal to the native host converter (csrc/native/
jb_hostfv_wide.hpp) and to the Python converter (tests/test_fv_wide.py).

Global weights keep the converter's sequential semantics inside a batch:
datum i of a training batch sees the document counts after datums 0..i
were added (a sort by (feature, datum) gives each datum's df at its own
position), then the table advances by the whole batch (index_add_ in HBM).
The table is the WeightManager's (fv_converter/converter.py): DeviceDf keeps
the HBM copy authoritative while GPU batches run and hands it back to the
host arrays when host code reads them (MIX, save, host conversion).
"""
from __future__ import annotations

import numpy as np
import torch

from . import hip


class DeviceDf:
    """HBM copy of a WeightManager's df / diff arrays (counts stay on the host)"""

    def __init__(self, wm, device):
        self.wm = wm
        self.device = device
        self.df = None
        self.diff = None
        self.dev_valid = False      # device copy current
        self.host_valid = True      # host copy current

    def push(self) -> None:
        if self.dev_valid:
            return
        wm = self.wm
        if wm.df is None:
            wm.df = np.zeros(wm.H, np.int64)
            wm.diff = np.zeros(wm.H, np.int64)
        self.df = torch.from_numpy(wm.df).to(self.device)
        self.diff = torch.from_numpy(wm.diff).to(self.device)
        self.dev_valid = True

    def device_changed(self) -> None:
        self.host_valid = False

    def pull(self, wm) -> None:
        if self.host_valid or self.df is None:
            return
        self.host_valid = True             # (before the copies: arrays() re-enters)
        wm.df[:] = self.df.cpu().numpy()
        wm.diff[:] = self.diff.cpu().numpy()

    def host_changed(self) -> None:
        self.dev_valid = False

    def clear(self) -> None:
        if self.df is not None:
            self.df.zero_()
            self.diff.zero_()
        self.host_valid = True


class WideDevice:
    def __init__(self, conv, device):
        from ..fv_converter.gpu_path import WideRuleTable
        rt = WideRuleTable(conv)
        self.conv = conv
        self.rt = rt
        self.device = torch.device(device)
        d = self.device
        self.srules = torch.from_numpy(rt.srules).to(d)
        self.nrules = torch.from_numpy(rt.nrules).to(d)
        self.crules = torch.from_numpy(rt.crules).to(d)
        self.blob = torch.from_numpy(rt.blob).to(d)
        self.H = rt.H
        self.err = torch.zeros(1, dtype=torch.int32, device=d)
        self.name_bytes = int(hip.fvw_name_bytes())
        self.df = None
        if conv.uses_global_weight:
            self.df = DeviceDf(conv.weights, d)
            conv.weights.device_table = self.df

    def convert(self, buf, buf_len: int, datum_off, datum_len, n: int, update: bool):
        """-> (row_ptr [n + 1] int64, idx, val, total slots) on the device"""
        d = self.device
        rt = self.rt
        base = torch.empty(max(n, 1), dtype=torch.int64, device=d)
        tot = torch.empty(max(n, 1), dtype=torch.int64, device=d)
        hip.fvw_count(buf, buf_len, datum_off, datum_len, n, self.srules, rt.n_srules, self.nrules,
                      rt.n_nrules, rt.n_crules, self.blob, base, tot, self.err)
        row_ptr = torch.zeros(n + 1, dtype=torch.int64, device=d)
        if n:
            torch.cumsum(tot[:n], 0, out=row_ptr[1:])
        total = int(row_ptr[n].item())
        cap = max(total, 1)
        idx = torch.empty(cap, dtype=torch.int32, device=d)
        val = torch.empty(cap, dtype=torch.float32, device=d)
        hs = torch.empty(cap, dtype=torch.int64, device=d)
        names = torch.empty(cap * self.name_bytes, dtype=torch.uint8, device=d)
        # zero: the combination region is written only after the weights pass,
        # which must not read its (not yet written) slots
        gw = torch.zeros(cap, dtype=torch.uint8, device=d)
        hip.fvw_emit(buf, buf_len, datum_off, datum_len, n, row_ptr, self.srules, rt.n_srules,
                     self.nrules, rt.n_nrules, self.blob, self.H, idx, val, hs, names, gw, self.err)
        if self.df is not None:
            self._weigh(row_ptr, total, n, idx, val, gw, update)
        if rt.n_crules:
            hip.fvw_comb(buf, n, row_ptr, base, self.srules, self.nrules, self.crules,
                         rt.n_crules, self.blob, self.H, idx, val, hs, names)
        return row_ptr, idx, val, total

    def _weigh(self, row_ptr, total: int, n: int, idx, val, gw, update: bool) -> None:
        """idf / bm25 on the slots of global-weighted rules (converter.py
        _convert semantics, datum by datum within the batch): one HIP launch
        chain (csrc/hip/df.hip), the table advanced in HBM"""
        wm = self.conv.weights
        self.df.push()
        N0, L0 = int(wm.counts[0]), int(wm.counts[1])
        if n == 0:
            return
        sel_len = torch.zeros(1, dtype=torch.int64, device=self.device)
        hip.df_weigh(row_ptr, n, total, idx, val, gw, self.df.df, self.df.diff, N0, L0, update, sel_len)
        if update:
            self.df.device_changed()
            tl = int(sel_len.item())
            wm.counts[0] += n
            wm.counts[2] += n
            wm.counts[1] += tl
            wm.counts[3] += tl
