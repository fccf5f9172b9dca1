"""Python mirror of the reference's reduction compute stage.

``reduce`` is one registered compute launched once (source/compute.h:90-91);
``Compute`` mirrors ``HiCCL::Compute<T>`` (source/compute.h:26-204):
``add`` / ``start`` / ``wait`` / ``report`` / ``measure`` with the same
argument meaning.  Both call straight into the HIP library through the C ABI
(include/hiccl_reduce.h); device memory and streams come from torch.
"""
import ctypes

import torch

from . import _lib as L


def _stream_handle(stream, device=None):
    if stream is None:
        return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
    if isinstance(stream, int):
        return ctypes.c_void_p(stream)
    return ctypes.c_void_p(stream.cuda_stream)


def _ptr_table(ptrs):
    t = (ctypes.c_void_p * max(1, len(ptrs)))()
    for k, p in enumerate(ptrs):
        t[k] = p
    return t


def _dtype_code(t):
    try:
        return L.DTYPE_OF_TORCH[t.dtype]
    except KeyError:
        raise TypeError(f"hiccl: unsupported dtype {t.dtype}") from None


def _check_tensor(t, what):
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"hiccl: {what} must be a torch.Tensor")
    if not t.is_cuda:
        raise ValueError(f"hiccl: {what} must be a device tensor (the HIP path has no CPU mode)")
    if not t.is_contiguous():
        raise ValueError(f"hiccl: {what} must be contiguous")


def reduce(out, inputs, count=None, stream=None, config=None):
    """out[:count] = ((0 + inputs[0]) + inputs[1]) + ... in the list order.

    Mirrors one compute of compute.h: inputs are summed in list order with
    the accumulator starting at 0 in the element type.  ``out`` may be one
    of the inputs (in place).  Asynchronous on ``stream`` (default: torch's
    current stream).  ``config``: dict of hiccl_reduce_config_t fields.
    """
    _check_tensor(out, "out")
    if count is None:
        count = out.numel()
    if count < 0:
        raise ValueError(f"hiccl: count={count} < 0")
    dt = _dtype_code(out)
    ptrs = []
    for k, x in enumerate(inputs):
        _check_tensor(x, f"inputs[{k}]")
        if x.device != out.device:
            raise ValueError(f"hiccl: inputs[{k}] is on {x.device}, out on {out.device}")
        if x.dtype != out.dtype:
            raise TypeError(f"hiccl: inputs[{k}] dtype {x.dtype} != out dtype {out.dtype}")
        if x.numel() < count:
            raise ValueError(f"hiccl: inputs[{k}] has {x.numel()} < count={count} elements")
        ptrs.append(x.data_ptr())
    if out.numel() < count:
        raise ValueError(f"hiccl: out has {out.numel()} < count={count} elements")
    tab = _ptr_table(ptrs)
    with torch.cuda.device(out.device):  # the library launches on the current device
        s = _stream_handle(stream, out.device)
        if config is None:
            rc = L.lib().hiccl_reduce(dt, ctypes.c_void_p(out.data_ptr()), tab, len(ptrs), count, s)
        else:
            cfg = L.ReduceConfig(**config)
            rc = L.lib().hiccl_reduce_ex(dt, ctypes.c_void_p(out.data_ptr()), tab, len(ptrs), count, s,
                                         ctypes.byref(cfg))
    L.check(rc, "hiccl_reduce")
    return out


def reduce_ptrs(dtype_code, out_ptr, in_ptrs, count, stream=None, config=None):
    """Raw-pointer form (pointers already offset), used by the Comm layer."""
    tab = _ptr_table(list(in_ptrs))
    s = _stream_handle(stream)
    if config is None:
        rc = L.lib().hiccl_reduce(dtype_code, ctypes.c_void_p(out_ptr), tab, len(in_ptrs), count, s)
    else:
        cfg = L.ReduceConfig(**config)
        rc = L.lib().hiccl_reduce_ex(dtype_code, ctypes.c_void_p(out_ptr), tab, len(in_ptrs), count, s,
                                     ctypes.byref(cfg))
    L.check(rc, "hiccl_reduce")


def bucket(n, count, dtype=torch.float32, device=None):
    """A reduction bucket in the library's layout (hiccl_bucket_alloc): n
    inputs and one output of ``count`` elements carved from ONE device
    allocation, buffer j at j x hiccl_bucket_stride (the buffer rounded up to
    64 KiB, plus 64 KiB), so the n + 1 streams keep one fixed relative
    placement.  The slab comes from torch's allocator
    (one hipMalloc for a fresh large block) and lives as long as any view.
    Returns (inputs, output): contiguous 1-D views."""
    esz = torch.empty((), dtype=dtype).element_size()
    stride = L.lib().hiccl_bucket_stride(L.DTYPE_OF_TORCH.get(dtype, -1), count)
    if not stride:
        raise ValueError(f"hiccl: no bucket layout for dtype {dtype}, count {count}")
    assert stride % esz == 0
    se = stride // esz
    slab = torch.empty((n + 1) * se, dtype=dtype, device=device if device is not None else "cuda")
    views = [slab[j * se:j * se + count] for j in range(n + 1)]
    return views[:n], views[n]


def auto_choice(dtype, count, n, config=None, cus=256):
    """What a one-shot call (and a one-compute plan at TILE unroll 2 / 4 or
    AUTO) resolves to on a GPU of ``cus`` CUs, without a device:
    ``hiccl_reduce_auto_choice_ex``.  ``dtype``: a torch dtype or an
    HICCL_* code; ``n`` may be a plan's packet-weighted mean.  Returns a dict
    with engine, unroll, blocks_per_cu, dynamic and store_policy (2 nt, 4
    write-through); raises HicclError for a config no kernel has."""
    dt = L.DTYPE_OF_TORCH[dtype] if isinstance(dtype, torch.dtype) else int(dtype)
    cfg = ctypes.byref(L.ReduceConfig(**config)) if config else None
    out = [ctypes.c_int() for _ in range(5)]
    rc = L.lib().hiccl_reduce_auto_choice_ex(dt, cfg, count, float(n), cus, *[ctypes.byref(v) for v in out])
    L.check(rc, "hiccl_reduce_auto_choice_ex")
    return dict(zip(("engine", "unroll", "blocks_per_cu", "dynamic", "store_policy"), (v.value for v in out)))


class Compute:
    """``HiCCL::Compute<T>`` (source/compute.h:26-204) on the batched plan.

    add(inputbuf, outputbuf, count, compid)  compute.h:47-85 -- records the
        compute only when ``myid == compid`` (SPMD: every rank calls add).
        ``inputbuf`` is a list of tensors or (tensor, element_offset) pairs,
        ``outputbuf`` a tensor or (tensor, element_offset).
    start()   compute.h:87-106 -- ONE batched kernel for all computes.
    wait()    compute.h:107-117.
    report()  compute.h:119-135 (local numbers; the Comm layer gathers).
    measure(warmup, numiter[, count])  compute.h:137-203.
    """

    def __init__(self, dtype=torch.float32, device=None, myid=0, acc=L.HICCL_ACC_NATIVE,
                 engine=L.HICCL_ENGINE_AUTO, config=None):
        self.dtype = dtype
        self.code = L.DTYPE_OF_TORCH[dtype]
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        self.myid = myid
        self.numcomp = 0
        self.inputbuf = []
        self.outputbuf = []
        self.count = []
        self._keep = []  # keep tensors alive while registered
        h = ctypes.c_void_p()
        L.check(L.lib().hiccl_reduce_plan_create(ctypes.byref(h), self.code, device), "plan_create")
        self._plan = h
        if acc != L.HICCL_ACC_NATIVE:
            L.check(L.lib().hiccl_reduce_plan_set_acc(self._plan, acc), "plan_set_acc")
        if engine != L.HICCL_ENGINE_AUTO:
            L.check(L.lib().hiccl_reduce_plan_set_engine(self._plan, engine), "plan_set_engine")
        if config is not None:
            self.set_config(config)

    def set_config(self, config):
        """Kernel configuration of the plan (dict of hiccl_reduce_config_t
        fields; hiccl_reduce_plan_set_config).  A field the plan kernels do
        not honour raises HicclError."""
        cfg = L.ReduceConfig(**config)
        L.check(L.lib().hiccl_reduce_plan_set_config(self._plan, ctypes.byref(cfg)), "plan_set_config")

    def set_peer(self, flags):
        """Peer-memory policy of the plan's launches (hiccl_reduce_plan_set_peer):
        HICCL_PEER_STORES (outputs in another GPU's memory: system-scope
        write-through stores) | HICCL_PEER_LOADS (inputs there: system-scope
        loads).  Same results."""
        L.check(L.lib().hiccl_reduce_plan_set_peer(self._plan, flags), "plan_set_peer")

    def peer(self):
        return L.lib().hiccl_reduce_plan_peer(self._plan)

    def store_policy(self):
        """The store form of the plan's launches (hiccl_reduce_plan_store_policy):
        2 nt, 4 system-scope write-through."""
        return L.lib().hiccl_reduce_plan_store_policy(self._plan)

    def engine(self):
        """Engine the last upload resolved to (HICCL_ENGINE_TILE / _PHASE)."""
        return L.lib().hiccl_reduce_plan_engine(self._plan)

    @staticmethod
    def _ptr(buf, esz):
        if isinstance(buf, tuple):
            t, off = buf
        else:
            t, off = buf, 0
        return t, t.data_ptr() + off * esz

    def add(self, inputbuf, outputbuf, count, compid):
        if self.myid != compid:
            return
        esz = L.lib().hiccl_dtype_size(self.code)
        ins = [self._ptr(b, esz) for b in inputbuf]
        ot, op = self._ptr(outputbuf, esz)
        tab = _ptr_table([p for _, p in ins])
        L.check(L.lib().hiccl_reduce_plan_add(self._plan, ctypes.c_void_p(op), tab, len(ins), count),
                "plan_add")
        self._keep.append((ot, [t for t, _ in ins]))
        self.inputbuf.append([p for _, p in ins])
        self.outputbuf.append(op)
        self.count.append(count)
        self.numcomp += 1

    def stream_handle(self):
        """The plan's own stream (hipStream_t as int)."""
        return L.lib().hiccl_reduce_plan_stream(self._plan)

    def start(self, stream=None, each=False):
        """Launch on ``stream`` (torch stream or raw handle); default = the
        plan's own stream (the reference keeps one per compute, compute.h:76-78),
        ordered after the work already queued on torch's current stream (the
        inputs it produced), so no synchronisation is needed first."""
        if stream is None:
            own = torch.cuda.ExternalStream(self.stream_handle(), device=self.device)
            own.wait_stream(torch.cuda.current_stream(self.device))
            s = ctypes.c_void_p(self.stream_handle())
        else:
            s = _stream_handle(stream, self.device)
        fn = L.lib().hiccl_reduce_plan_launch_each if each else L.lib().hiccl_reduce_plan_launch
        L.check(fn(self._plan, s), "plan_launch")

    def enqueue(self, stream=None):
        """Launch on ``stream`` (default torch's current stream) without
        remembering it for :meth:`wait` (hiccl_reduce_plan_enqueue): for
        stream-ordered pipelines that synchronise the stream themselves."""
        L.check(L.lib().hiccl_reduce_plan_enqueue(self._plan, _stream_handle(stream, self.device)), "plan_enqueue")

    def wait(self):
        L.check(L.lib().hiccl_reduce_plan_sync(self._plan), "plan_sync")

    def bytes(self):
        """Sum of count * (n + 1) * sizeof(T) (compute.h:197-203)."""
        return L.lib().hiccl_reduce_plan_bytes(self._plan)

    def report(self):
        numinput = sum(len(x) for x in self.inputbuf)
        return f"numcomp: {self.numcomp}({numinput})"

    def measure(self, warmup, numiter, count=None, each=False):
        """Time start()+wait() like compute.h:137-196; returns the stats dict.

        ``count`` is the element count the GB/s figure is priced on
        (compute.h:188); default = the two-argument overload's
        sum of count*(n+1) (compute.h:197-203), i.e. reads + writes.
        """
        import time
        data = (self.bytes() if count is None else count * torch.tensor([], dtype=self.dtype).element_size())
        times = []
        for it in range(-warmup, numiter):
            torch.cuda.synchronize(self.device)
            t0 = time.perf_counter()
            self.start(each=each)
            self.wait()
            t = time.perf_counter() - t0
            if it >= 0:
                times.append(t)
        times.sort()
        avg = sum(times) / len(times)
        stats = {"min": times[0], "median": times[len(times) // 2], "max": times[-1], "avg": avg,
                 "data": data}
        for k in ("min", "median", "max", "avg"):
            stats[k + "_GBps"] = data / stats[k] / 1e9
        return stats

    def close(self):
        if self._plan:
            L.lib().hiccl_reduce_plan_destroy(self._plan)
            self._plan = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Program:
    """A program (include/hiccl_reduce.h ``hiccl_program_*``): signal/wait
    phases folded into the launch of one batch of independent computes --
    the phases run first (one wave, in order), the units after the last
    phase.  HiCCL::Comm records its stream-ordered pipeline as programs.

    add_signal(sig_ptrs, wait_ptrs)   one phase (device flag addresses),
                                      before the first add_plan.
    add_plan(compute)                 the computes a :class:`Compute` holds
                                      now (its dtype must be the program's,
                                      or torch.uint8 = exact byte copies).
    launch(epochs, epoch_dev, err, timeout_s, stream)
    """

    def __init__(self, dtype=torch.float32, device=None):
        if device is None:
            device = torch.cuda.current_device()
        self.device = device
        h = ctypes.c_void_p()
        L.check(L.lib().hiccl_program_create(ctypes.byref(h), L.DTYPE_OF_TORCH[dtype], device), "program_create")
        self._prog = h
        self._keep = []

    def add_signal(self, sig_ptrs, wait_ptrs):
        st, wt = _ptr_table(list(sig_ptrs)), _ptr_table(list(wait_ptrs))
        L.check(L.lib().hiccl_program_add_signal(self._prog, st, len(sig_ptrs), wt, len(wait_ptrs)),
                "program_add_signal")

    def add_plan(self, compute):
        L.check(L.lib().hiccl_program_add_plan(self._prog, compute._plan), "program_add_plan")
        self._keep.append(compute)

    def set_max_workgroups(self, n):
        """Cap the launch at ``n`` workgroups (0: the default)."""
        L.check(L.lib().hiccl_program_set_max_workgroups(self._prog, int(n)), "program_set_max_workgroups")

    def units(self):
        return L.lib().hiccl_program_num_units(self._prog)

    def phases(self):
        return L.lib().hiccl_program_num_phases(self._prog)

    def launch(self, epochs=(), epoch_dev=None, err=None, timeout_s=10.0, stream=None):
        ep = (ctypes.c_uint32 * max(1, len(epochs)))(*epochs)
        L.check(L.lib().hiccl_program_launch(self._prog, ep, ctypes.c_void_p(epoch_dev or 0),
                                             ctypes.c_void_p(err or 0), float(timeout_s),
                                             _stream_handle(stream, self.device)), "program_launch")

    def close(self):
        if self._prog:
            L.lib().hiccl_program_destroy(self._prog)
            self._prog = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostPipe:
    """Host-resident buckets (include/hiccl_reduce.h hiccl_host_pipe_*):
    ``reduce(out, inputs)`` sums host tensors in list order on the GPU,
    staging ``chunk_bytes`` per input through device memory with H2D /
    kernel / D2H pipelined over ``depth`` streams.  Blocking; same bits as
    :func:`reduce`.  Pin the tensors (``pin_memory()``) for the overlap."""

    def __init__(self, dtype=torch.float32, device=None, chunk_bytes=0, depth=0):
        self.dtype = dtype
        self.code = L.DTYPE_OF_TORCH[dtype]
        if device is None:
            device = torch.cuda.current_device()
        h = ctypes.c_void_p()
        L.check(L.lib().hiccl_host_pipe_create(ctypes.byref(h), self.code, device, chunk_bytes, depth),
                "host_pipe_create")
        self._pipe = h

    def reduce(self, out, inputs, count=None):
        for k, t in enumerate([out] + list(inputs)):
            what = "out" if k == 0 else f"inputs[{k - 1}]"
            if not isinstance(t, torch.Tensor) or t.is_cuda:
                raise ValueError(f"hiccl: {what} must be a host tensor (HostPipe stages it to the GPU)")
            if not t.is_contiguous():
                raise ValueError(f"hiccl: {what} must be contiguous")
            if t.dtype != self.dtype:
                raise TypeError(f"hiccl: {what} dtype {t.dtype} != pipe dtype {self.dtype}")
        if count is None:
            count = out.numel()
        if any(t.numel() < count for t in [out] + list(inputs)):
            raise ValueError(f"hiccl: a buffer has fewer than count={count} elements")
        tab = _ptr_table([t.data_ptr() for t in inputs])
        L.check(L.lib().hiccl_host_pipe_reduce(self._pipe, ctypes.c_void_p(out.data_ptr()), tab,
                                               len(inputs), count), "host_pipe_reduce")
        return out

    def close(self):
        if self._pipe:
            L.lib().hiccl_host_pipe_destroy(self._pipe)
            self._pipe = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def fill_uniform(t, seed, k, first=0, stream=None):
    """Synthetic input k: uniform [-1,1) of hash(seed, k, first + i) (matches the oracle)."""
    _check_tensor(t, "t")
    L.check(L.lib().hiccl_fill_uniform(_dtype_code(t), ctypes.c_void_p(t.data_ptr()), t.numel(),
                                       seed, k, first, _stream_handle(stream)), "fill_uniform")
    return t


def stream_copy(dst, src, nbytes=None, stream=None):
    """Plain 16-B/lane device copy (the achievable-bandwidth ceiling)."""
    if nbytes is None:
        nbytes = src.numel() * src.element_size()
    L.check(L.lib().hiccl_stream_copy(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                      nbytes, _stream_handle(stream)), "stream_copy")
