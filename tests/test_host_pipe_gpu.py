"""GPU tier: host-resident buckets through hiccl_host_pipe_* (SURVEY.md 8f
row 4) vs the oracle, bit-exact: pinned and pageable host memory, chunking
(partial last chunk, chunk sizes that are not a multiple of the element),
pipeline depths 1-8, n = 0 / 1 / many / > 64 (device pointer table),
misaligned host pointers, in place into input 0, and the device path's bits
on a multi-chunk bucket."""
import numpy as np
import pytest
import torch

import hiccl_amd
from conftest import bits_equal, first_mismatch

pytestmark = pytest.mark.gpu

NP_OF = {torch.float32: np.float32, torch.float64: np.float64, torch.bfloat16: np.uint16}


def host_tensor(a, dtype, pinned, offset=0):
    """Host tensor holding numpy rows `a`, `offset` elements into its buffer."""
    if dtype == torch.bfloat16:
        t = torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
    else:
        t = torch.from_numpy(a.copy())
    buf = torch.empty(t.numel() + offset + 4, dtype=dtype)
    if pinned:
        buf = buf.pin_memory()
    view = buf[offset:offset + t.numel()]
    view.copy_(t)
    return view


def as_np(t):
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


@pytest.mark.parametrize("pinned", [True, False], ids=["pinned", "pageable"])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16, torch.float64], ids=["f32", "bf16", "f64"])
@pytest.mark.parametrize("n", [0, 1, 3, 8, 70])
def test_host_pipe_matches_oracle(oracle, pinned, dtype, n):
    count = 100_003
    np_dt = NP_OF[dtype]
    x = oracle.fill(n, count, seed=17 + n, dtype=np_dt) if n else np.zeros((0, count), np_dt)
    exp = oracle.reduce(list(x), count=count, dtype=np_dt)
    ins = [host_tensor(x[k], dtype, pinned, offset=k % 3) for k in range(n)]
    for chunk_bytes, depth in ((0, 0), (40_002, 1), (65536, 2), (3 * 4096 + 6, 8)):
        pipe = hiccl_amd.HostPipe(dtype, device=0, chunk_bytes=chunk_bytes, depth=depth)
        out = host_tensor(np.zeros(count, np_dt), dtype, pinned, offset=1)
        pipe.reduce(out, ins)
        got = as_np(out)
        assert bits_equal(got, exp), f"chunk={chunk_bytes} depth={depth}: {first_mismatch(got, exp)}"
        pipe.close()


def test_host_pipe_in_place_and_reuse(oracle):
    """out == inputs[0] (exact aliasing), and one pipe reused for growing n."""
    pipe = hiccl_amd.HostPipe(torch.float32, device=0, chunk_bytes=1 << 16, depth=3)
    for n in (2, 5, 9):
        count = 77_777
        x = oracle.fill(n, count, seed=n)
        exp = oracle.reduce(list(x))
        ins = [host_tensor(x[k], torch.float32, True) for k in range(n)]
        pipe.reduce(ins[0], ins)
        assert bits_equal(ins[0].numpy(), exp)
    pipe.close()


def test_host_pipe_same_bits_as_device_path():
    """8 inputs x 2^25 f32 (two default 64 MiB chunks + the pipeline
    wrap-around at depth 3 with 16 MiB chunks): host pipe == hiccl_reduce."""
    n, count = 8, 1 << 25
    dev_in = [torch.empty(count, device="cuda:0") for _ in range(n)]
    for k, t in enumerate(dev_in):
        hiccl_amd.fill_uniform(t, 2024, k)
    dev_out = torch.empty(count, device="cuda:0")
    hiccl_amd.reduce(dev_out, dev_in)
    host_in = [t.cpu().pin_memory() for t in dev_in]
    expect = dev_out.cpu()
    for chunk_bytes in (0, 16 << 20):
        pipe = hiccl_amd.HostPipe(torch.float32, device=0, chunk_bytes=chunk_bytes)
        out = torch.empty(count).pin_memory()
        pipe.reduce(out, host_in)
        assert torch.equal(out.view(torch.int32), expect.view(torch.int32))
        pipe.close()


def test_host_pipe_refuses_device_tensors_and_bad_args():
    pipe = hiccl_amd.HostPipe(torch.float32, device=0)
    d = torch.zeros(8, device="cuda:0")
    with pytest.raises(ValueError, match="host tensor"):
        pipe.reduce(d, [d])
    h = torch.zeros(16)
    with pytest.raises(hiccl_amd.HicclError, match="overlap"):
        pipe.reduce(h[1:9], [h[0:8]])
    pipe.close()
