"""Per-kernel roofline ledger: every C-ABI launch of csu goes through ``launch()``, which names the
call and states its ALGORITHMIC work (FLOPs; bytes = each input read once + each output written
once).  While a ``KernelLedger`` is active, each launch is timed with HIP events on its own stream.
Eager mode: idempotent launches are re-run ``repeat`` times back-to-back between the two events
(the per-event overhead then stays out of the per-launch time), non-idempotent ones (the in-place
AdamW) are timed once; the repeats find their inputs in the caches, so memory-bound kernels read
up to ~12 % faster than inside the step.  Graph mode (``graph=True``): the launches of a stream
capture are bracketed by external HIP event-record nodes, so each replay of the captured step
times every kernel where it really runs (bench.py's single-process roofline); a bracket adds the
launch's dispatch and completion (~2-5 us per launch against the rocprofv3 kernel time: 5 % on the
attention backward, 16 % on the 14-us token GEMMs), so graph-mode fractions err low.  ``summary()`` gives, per call name, launches, measured time,
achieved GB/s / TFLOP/s, the roofline time t_roof = max(FLOPs / P_mfma, bytes / BW_hbm) and the
fraction t_roof / t_measured (MI355X_MICROARCH.md peaks: HBM 8 TB/s, dense bf16 MFMA 2.5 PF/s,
fp32 MFMA 157.3 TF/s)."""
from __future__ import annotations

import collections
import ctypes
from typing import Callable, Dict, List, Optional

import torch

from ._lib import check

HBM_GBS = 8000.0
PEAK_TFLOPS = {"bf16": 2500.0, "f32": 157.3, "fp8": 5000.0}

_ACTIVE: Optional["KernelLedger"] = None


class _HipEvent:
    """A HIP timing event recorded with hipEventRecordExternal (csu_event_record_ext): inside a stream
    capture it is an event-record node of the graph, re-stamped by every replay."""

    def __init__(self):
        from ._lib import lib
        self._lib = lib()
        h = ctypes.c_void_p()
        check(self._lib.csu_event_create(ctypes.byref(h)), "event_create")
        self.h = h

    def record(self):
        check(self._lib.csu_event_record_ext(self.h, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
              "event_record_ext")

    def elapsed_time(self, end: "_HipEvent") -> float:
        ms = ctypes.c_float()
        check(self._lib.csu_event_elapsed_ms(self.h, end.h, ctypes.byref(ms)), "event_elapsed_ms")
        return float(ms.value)

    def __del__(self):
        try:
            self._lib.csu_event_destroy(self.h)
        except Exception:
            pass


class KernelLedger:
    """``graph=False``: time the launches of eager steps (idempotent ones repeated ``repeat`` times).
    ``graph=True``: only launches made while a stream is being captured are recorded, each bracketed
    by two external HIP event nodes inside the graph; call ``collect()`` after each replay of that
    graph (synchronized) -- ``summary()`` then averages every launch over the collected replays, i.e.
    the kernels' times as they run inside the replayed step (inputs left in the caches, or dirty, by
    the kernel before: what rocprofv3 sees over the timed region)."""

    def __init__(self, repeat: int = 4, graph: bool = False):
        self.repeat = max(1, int(repeat))
        self.graph = bool(graph)
        self.rows: List[tuple] = []
        self._acc: List[float] = []
        self.replays = 0

    def collect(self):
        """Add the event-pair times of the replay that just finished (graph mode)."""
        torch.cuda.synchronize()
        if len(self._acc) < len(self.rows):
            self._acc += [0.0] * (len(self.rows) - len(self._acc))
        for i, r in enumerate(self.rows):
            self._acc[i] += r[1].elapsed_time(r[2])
        self.replays += 1

    def __enter__(self):
        global _ACTIVE
        self._prev, _ACTIVE = _ACTIVE, self
        return self

    def __exit__(self, *exc):
        global _ACTIVE
        _ACTIVE = self._prev
        return False

    def launches(self) -> List[Dict]:
        """Every recorded launch in order: name, shape tag, measured us, algorithmic bytes / FLOPs."""
        torch.cuda.synchronize()
        out = []
        for i, (name, e0, e1, reps, flops, nbytes, prec, tag) in enumerate(self.rows):
            ms = self._acc[i] / self.replays if self.graph else e0.elapsed_time(e1) / reps
            out.append({"kernel": name, "tag": tag, "us": round(ms * 1e3, 2), "bytes": int(nbytes), "flops": int(flops)})
        return out

    def summary(self, steps: int = 1) -> List[Dict]:
        """Per call name (sorted by measured time): launches per step, avg us per launch, algorithmic
        bytes / FLOPs per launch, achieved GB/s and TFLOP/s, bound, t_roof and frac."""
        torch.cuda.synchronize()
        agg = collections.OrderedDict()
        if self.graph and not self.replays:
            raise RuntimeError("KernelLedger(graph=True): collect() after at least one replay")
        for i, (name, e0, e1, reps, flops, nbytes, prec, _) in enumerate(self.rows):
            a = agg.setdefault(name, {"n": 0, "ms": 0.0, "flops": 0.0, "bytes": 0.0, "prec": prec})
            a["n"] += 1
            a["ms"] += self._acc[i] / self.replays if self.graph else e0.elapsed_time(e1) / reps
            a["flops"] += flops
            a["bytes"] += nbytes
        out = []
        for name, a in agg.items():
            n = a["n"]
            us = a["ms"] / n * 1e3
            peak = PEAK_TFLOPS[a["prec"]]
            t_mem = a["bytes"] / n / (HBM_GBS * 1e9) * 1e6           # us
            t_mma = a["flops"] / n / (peak * 1e12) * 1e6
            t_roof = max(t_mem, t_mma)
            out.append({"kernel": name, "launches_per_step": round(n / steps, 2), "avg_us": round(us, 2),
                        "us_per_step": round(us * n / steps, 1),
                        "bytes_per_launch": int(a["bytes"] / n), "flops_per_launch": int(a["flops"] / n),
                        "achieved_GBs": round(a["bytes"] / n / (us * 1e-6) / 1e9, 1),
                        "achieved_TFLOPs": round(a["flops"] / n / (us * 1e-6) / 1e12, 2),
                        "bound": "hbm" if t_mem >= t_mma else "mfma", "precision": a["prec"],
                        "t_roof_us": round(t_roof, 3), "frac": round(t_roof / us, 4) if us > 0 else None})
        out.sort(key=lambda r: -r["us_per_step"])
        return out


def launch(name: str, fn: Callable[[], int], flops: float = 0.0, nbytes: float = 0.0, idem: bool = True,
           prec: str = "bf16", tag: str = ""):
    """Run ``fn`` (a C-ABI call returning its status code) and check it; time it when a ledger is
    active.  ``idem``: the call can be repeated without changing its result (outputs overwritten
    from unchanged inputs)."""
    led = _ACTIVE
    capturing = torch.cuda.is_current_stream_capturing()
    if led is None or capturing != led.graph:
        check(fn(), name)
        return
    if capturing:   # graph mode: event-record nodes around the launch, re-stamped by every replay
        e0, e1 = _HipEvent(), _HipEvent()
        e0.record()
        check(fn(), name)
        e1.record()
        led.rows.append((name, e0, e1, 1, float(flops), float(nbytes), prec, tag))
        return
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if idem:
        check(fn(), name)
        e0.record()
        for _ in range(led.repeat):
            check(fn(), name)
        e1.record()
        reps = led.repeat
    else:
        e0.record()
        check(fn(), name)
        e1.record()
        reps = 1
    led.rows.append((name, e0, e1, reps, float(flops), float(nbytes), prec, tag))


def esize(t) -> int:
    return 0 if t is None else t.element_size()


def prec_of(t) -> str:
    return "f32" if t is not None and t.dtype == torch.float32 else "bf16"
