"""Allocation-placement probe (round 6): config 2's kernel time moves by up
to 8 % between buckets of one process (profiles/r06b_order.jsonl: 1.4623 /
1.5802 / 1.4788 ms), i.e. with the physical pages a bucket gets.  Is one
buffer the slow one, and does the allocation form change the spread?

Forms: `torch` (torch.empty per buffer: the caching allocator over
hipMalloc, as bench.py), `hipmalloc` (hipMalloc per buffer), `contig`
(hipExtMallocWithFlags(hipDeviceMallocContiguous) per buffer), `pool` (one
hipMalloc of 9 GiB carved at 1 GiB stride).  Every bucket stays allocated;
config 2 timed in interleaved rounds over all buckets; then, per buffer,
tools/libhbm_probe.so's read-only (inputs) / write-only (output) kernel
alone on that buffer.  One JSON line per bucket, then a summary.
  usage: python tools/alloc_probe.py [--buckets 3] [--rounds 4] [--reps 10] [--forms torch,hipmalloc,contig,pool]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import hiccl_amd  # noqa: E402
from hiccl_amd import _lib as L  # noqa: E402

N, COUNT, SEED = 8, 1 << 28, 1234  # --n / --log2count override
BYTES = COUNT * 4
HIP = ctypes.CDLL("libamdhip64.so.7")
HIP.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
HIP.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
HIP.hipFree.argtypes = [ctypes.c_void_p]
CONTIGUOUS = 0x4  # hipDeviceMallocContiguous


def hip_alloc(nbytes, flags=None):
    p = ctypes.c_void_p()
    rc = HIP.hipMalloc(ctypes.byref(p), nbytes) if flags is None else HIP.hipExtMallocWithFlags(
        ctypes.byref(p), nbytes, flags)
    if rc != 0 or not p.value:
        raise MemoryError(f"hip allocation of {nbytes} B (flags {flags}) failed: {rc}")
    return p.value


class Bucket:
    def __init__(self, form):
        self.form, self.keep, self.raw = form, [], []
        if form == "torch":
            ts = [torch.empty(COUNT, device="cuda") for _ in range(N + 1)]
            self.keep = ts
            ptrs = [t.data_ptr() for t in ts]
        elif form.startswith("pool"):
            # pool[c][+<extra KiB>][:desc][:outfirst]: one allocation, buffer j
            # at j x (1 GiB + extra); poolc: hipDeviceMallocContiguous; desc:
            # inputs in descending order; outfirst: the output at slot 0
            spec = form.split(":")
            contig = spec[0].startswith("poolc")
            head = spec[0][5:] if contig else spec[0][4:]
            extra = int(head[1:]) * 1024 if head.startswith("+") else 0
            stride = BYTES + extra
            if head.startswith("x"):  # poolx<k>: stride k/2 x the buffer + 64 KiB
                stride = int(head[1:]) * BYTES // 2 + (64 << 10)
            base = hip_alloc((N + 1) * stride, CONTIGUOUS if contig else None)
            self.raw = [base]
            slots = list(range(N + 1))
            if "outfirst" in spec:
                slots = slots[1:] + slots[:1]
            if "desc" in spec:
                slots = slots[:N][::-1] + slots[N:]
            ptrs = [base + j * stride for j in slots]
        else:
            ptrs = [hip_alloc(BYTES, CONTIGUOUS if form == "contig" else None) for _ in range(N + 1)]
            self.raw = ptrs
        self.ins, self.out = ptrs[:N], ptrs[N]
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for k, p in enumerate(self.ins):
            L.check(L.lib().hiccl_fill_uniform(L.HICCL_FLOAT32, ctypes.c_void_p(p), COUNT, SEED, k, 0, st), "fill")

    def reduce(self):
        hiccl_amd.reduce_ptrs(L.HICCL_FLOAT32, self.out, self.ins, COUNT)

    def free(self):
        for p in self.raw:
            HIP.hipFree(ctypes.c_void_p(p))
        self.keep = []


def timed(fn, reps):
    s = torch.cuda.current_stream()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in ev:
        a.record(s)
        fn()
        b.record(s)
    torch.cuda.synchronize()
    return [a.elapsed_time(b) for a, b in ev]


def buffer_rates(bk, probe, reps):
    """GB/s of the probe's read-only kernel on each input alone and its
    write-only kernel on the output alone (256 workgroups, tile order)."""
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    rates = []
    for k, p in enumerate(bk.ins + [bk.out]):
        mode = 1 if k < N else 2
        tab = (ctypes.c_void_p * 1)(p)
        fn = lambda: probe.probe_run(mode, 256, 4, 2, 2, 0, 256, tab, 1, ctypes.c_void_p(p), BYTES, st)  # noqa: E731
        timed(fn, 2)
        ms = timed(fn, reps)
        rates.append(round(BYTES / (np.median(ms) * 1e-3) / 1e9, 1))
    return rates


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--buckets", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--forms", default="torch,hipmalloc,contig,pool")
    ap.add_argument("--fragment", type=int, default=0, help="seed: fragment free device memory before allocating")
    ap.add_argument("--interleave", action="store_true", help="forms in round-robin allocation order")
    ap.add_argument("--n", type=int, default=8)
    ap.add_argument("--log2count", type=int, default=28)
    args = ap.parse_args()
    global N, COUNT, BYTES
    N, COUNT = args.n, 1 << args.log2count
    BYTES = COUNT * 4
    probe = ctypes.CDLL(os.path.join(ROOT, "tools", "libhbm_probe.so"))
    probe.probe_run.restype = ctypes.c_int
    probe.probe_run.argtypes = [ctypes.c_int] * 7 + [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p,
                                                     ctypes.c_uint64, ctypes.c_void_p]
    frag = []
    if args.fragment:
        # fragment the device's free memory first: allocate ~2/3 of it in
        # pieces of 96 MiB-1.5 GiB, free every other one (kept until the end)
        rng = np.random.default_rng(args.fragment)
        free_b, _ = torch.cuda.mem_get_info()
        total, pieces = 0, []
        while total < free_b * 2 // 3:
            nb = int(rng.integers(96, 1536)) << 20
            pieces.append(hip_alloc(nb))
            total += nb
        for k, p in enumerate(pieces):
            if k % 2:
                HIP.hipFree(ctypes.c_void_p(p))
            else:
                frag.append(p)
        print(json.dumps({"fragmented": True, "pieces": len(pieces), "held_GiB": round(total / 2 / 2**30, 1)}),
              flush=True)
    buckets = []
    forms = args.forms.split(",")
    order = ([f for _ in range(args.buckets) for f in forms] if args.interleave
             else [f for f in forms for _ in range(args.buckets)])
    for form in order:
        try:
            buckets.append(Bucket(form))
        except MemoryError as e:
            print(json.dumps({"form": form, "error": str(e)}), flush=True)
    torch.cuda.synchronize()
    ref = torch.empty(COUNT, device="cuda")
    hiccl_amd.reduce_ptrs(L.HICCL_FLOAT32, ref.data_ptr(), buckets[0].ins, COUNT)
    ms = [[] for _ in buckets]
    for bk in buckets:
        timed(bk.reduce, 2)
    for _ in range(args.rounds):
        for i, bk in enumerate(buckets):
            ms[i] += timed(bk.reduce, args.reps)
    res = []
    for i, bk in enumerate(buckets):
        out = torch.empty(COUNT, device="cuda")
        torch.cuda.synchronize()
        # same inputs (same generator and seed) in every bucket: every output equals bucket 0's
        ok = True
        hiccl_amd.reduce_ptrs(L.HICCL_FLOAT32, out.data_ptr(), bk.ins, COUNT)
        torch.cuda.synchronize()
        ok = bool(torch.equal(out.view(torch.int32), ref.view(torch.int32)))
        del out
        r = {"bucket": i, "form": bk.form, "kernel_ms_mean": round(float(np.mean(ms[i])), 4),
             "kernel_ms_min": round(float(np.min(ms[i])), 4),
             "frac_of_8TBs": round((N + 1) * BYTES / (np.mean(ms[i]) * 1e-3) / 8e12, 4),
             "buffer_GBps_read_inputs_then_write_output": buffer_rates(bk, probe, 5), "bit_exact": ok,
             "addresses_GiB": [round(p / 2**30, 3) for p in bk.ins + [bk.out]]}
        res.append(r)
        print(json.dumps(r), flush=True)
    summ = {}
    for form in args.forms.split(","):
        t = [r["kernel_ms_mean"] for r in res if r["form"] == form]
        if t:
            summ[form] = {"kernel_ms": t, "spread_max_over_min": round(max(t) / min(t), 4)}
    print(json.dumps({"summary": summ}), flush=True)
    for bk in buckets:
        bk.free()
    for p in frag:
        HIP.hipFree(ctypes.c_void_p(p))
    return 0


if __name__ == "__main__":
    sys.exit(main())
