"""Input placement experiment: 8 x 2^28 fp32 inputs carved from one pool at
stride (1 GiB + s) for several s; kernel time by HIP events.  Tests whether
power-of-two separation between the inputs costs HBM bandwidth."""
import json
import sys

import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__import__("os").path.abspath(__file__))))
import hiccl_amd  # noqa: E402

n, count = 8, 1 << 28
MiB = 1 << 20
def run(stride_bytes, out_sep=0, reps=20):
    stride = stride_bytes // 4
    pool = torch.empty(n * stride + count + out_sep // 4 + 1024, dtype=torch.float32, device="cuda")
    ins = [pool[k * stride:k * stride + count] for k in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, 1234, k)
    o0 = n * stride + out_sep // 4
    out = pool[o0:o0 + count]
    torch.cuda.synchronize()
    for _ in range(5):
        hiccl_amd.reduce(out, ins)
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(s); hiccl_amd.reduce(out, ins); b.record(s)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]
    del pool, ins, out
    torch.cuda.empty_cache()
    return ms

base = 1 << 30
cases = [("0", 0), ("128K", 128 << 10), ("256K", 256 << 10), ("512K", 512 << 10), ("768K", 768 << 10),
         ("1M+256K", MiB + (256 << 10)), ("1.5M", 3 * MiB // 2), ("4K", 4096), ("64K", 64 << 10), ("1M", MiB), ("2M", 2 * MiB), ("3M", 3 * MiB), ("4M", 4 * MiB),
         ("8M", 8 * MiB), ("17M", 17 * MiB), ("64M", 64 * MiB), ("70.3M", 73741824), ("6M+4K", 6 * MiB + 4096),
         ("128M", 128 * MiB), ("257M", 257 * MiB), ("512M", 512 * MiB),
         ("-1M", -MiB), ("-4M", -4 * MiB), ("-8M", -8 * MiB), ("-16M", -16 * MiB)]
if len(sys.argv) > 1:
    keep = set(sys.argv[1].split(","))
    cases = [c for c in cases if c[0] in keep]
for label, extra in cases:
    st = base + extra
    pool_pad = max(0, -extra) * n  # inputs may overlap (read-only); the output never does
    ms = run(st, out_sep=pool_pad)
    print(json.dumps({"stride_extra": label, "stride_bytes": st, "kernel_ms": round(ms, 4),
                      "GBps": round(9 * count * 4 / ms / 1e6, 1)}), flush=True)
# output displacement with inputs at exactly 1 GiB apart
for_outputs = len(sys.argv) <= 2
for label, osep in [("out+0", 0), ("out+1M", MiB), ("out+4M", 4 * MiB), ("out+8M", 8 * MiB)]:
    if not for_outputs:
        break
    ms = run(base, out_sep=osep)
    print(json.dumps({"inputs_stride": "1G", "output_extra": label, "kernel_ms": round(ms, 4),
                      "GBps": round(9 * count * 4 / ms / 1e6, 1)}), flush=True)


def run_separate(color_bytes, reps=20):
    """Separate allocations (as HiCCL::allocate / torch.empty give), input k
    viewed at byte offset k * color_bytes (allocation coloring)."""
    c = color_bytes // 4
    bufs = [torch.empty(count + n * c + 1024, dtype=torch.float32, device="cuda") for _ in range(n + 1)]
    ins = [bufs[k][k * c:k * c + count] for k in range(n)]
    for k, t in enumerate(ins):
        hiccl_amd.fill_uniform(t, 1234, k)
    out = bufs[n][n * c:n * c + count]
    torch.cuda.synchronize()
    for _ in range(5):
        hiccl_amd.reduce(out, ins)
    s = torch.cuda.current_stream()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(reps)]
    for a, b in evs:
        a.record(s); hiccl_amd.reduce(out, ins); b.record(s)
    torch.cuda.synchronize()
    ms = sorted(a.elapsed_time(b) for a, b in evs)[reps // 2]
    ptrs = [hex(t.data_ptr()) for t in ins]
    del bufs, ins, out
    torch.cuda.empty_cache()
    return ms, ptrs


if len(sys.argv) > 3:
    for col in [int(v) for v in sys.argv[3].split(",")]:
        ms, ptrs = run_separate(col << 10)
        print(json.dumps({"separate_alloc_color_KiB": col, "kernel_ms": round(ms, 4),
                          "GBps": round(9 * count * 4 / ms / 1e6, 1), "ptrs": ptrs[:3]}), flush=True)
