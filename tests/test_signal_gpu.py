"""Stream-ordered signalling kernels (hiccl_signal_wait_dev /
hiccl_signal_wait_phases), single process: the flags live in this device's
memory, so every wait is satisfied by a signal of the same or an earlier
phase.  The cross-process protocol is covered by tests/test_mpi_gpu.py and
tests/test_c5_leg_gpu.py; these check the phase packing (more than 8 phases,
more than 64 flags), the epoch arithmetic (graph epoch counter, 32-bit wrap)
and the timeout path, which must set *err and return instead of hanging."""
import ctypes

import pytest
import torch

from hiccl_amd import _lib as L

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


class Phase(ctypes.Structure):
    _fields_ = [("sig", ctypes.c_void_p), ("nsig", ctypes.c_int),
                ("wait", ctypes.c_void_p), ("nwait", ctypes.c_int),
                ("epoch", ctypes.c_uint32)]


def _ptrs(flags, idx):
    return (ctypes.c_void_p * max(1, len(idx)))(*[flags.data_ptr() + 4 * i for i in idx])


def _stream():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _run(phases, flags, epoch_dev=None, timeout_s=5.0):
    """phases: [(sig_idx, wait_idx, epoch)] over the int32 flag tensor."""
    keep, arr = [], (Phase * len(phases))()
    for k, (si, wi, ep) in enumerate(phases):
        s, w = _ptrs(flags, si), _ptrs(flags, wi)
        keep += [s, w]
        arr[k] = Phase(ctypes.cast(s, ctypes.c_void_p), len(si), ctypes.cast(w, ctypes.c_void_p), len(wi), ep)
    err = torch.zeros(1, dtype=torch.int32, device=DEV)
    ed = ctypes.c_void_p(epoch_dev.data_ptr()) if epoch_dev is not None else None
    rc = L.lib().hiccl_signal_wait_phases(arr, len(phases), ed, ctypes.c_void_p(err.data_ptr()),
                                          ctypes.c_double(timeout_s), _stream())
    assert rc == 0, L.last_error()
    torch.cuda.synchronize()
    return int(err.item())


@pytest.mark.parametrize("nphase", [1, 8, 9, 20])
def test_phases_in_order(nphase):
    """Phase p signals flag p and waits for flags 0..p: satisfied only if the
    phases run in order (a later phase never waits for an unsignalled flag)."""
    flags = torch.zeros(32, dtype=torch.int32, device=DEV)
    phases = [([p], list(range(p + 1)), 100) for p in range(nphase)]
    assert _run(phases, flags) == 0
    assert flags[:nphase].tolist() == [100] * nphase
    assert not flags[nphase:].any()
    # epochs rising per phase: phase p re-signals 0..p with 200 + p
    phases = [(list(range(p + 1)), list(range(p + 1)), 200 + p) for p in range(nphase)]
    assert _run(phases, flags) == 0
    assert flags[:nphase].tolist() == [200 + nphase - 1] * nphase


def test_many_flags_one_phase():
    """More than 64 flags of a kind: all signalled before the first wait."""
    flags = torch.zeros(200, dtype=torch.int32, device=DEV)
    idx = list(range(150))
    assert _run([(idx, idx[::-1], 7)], flags) == 0
    assert flags[:150].tolist() == [7] * 150 and not flags[150:].any()


def test_mixed_packing():
    """Phases of 0..70 signal / wait flags, packed over several launches."""
    flags = torch.zeros(256, dtype=torch.int32, device=DEV)
    phases, base = [], 0
    for p, n in enumerate([0, 3, 64, 1, 70, 5, 0, 40, 33]):
        idx = list(range(base, base + n))
        phases.append((idx, idx, 11 + p))
        base += n
    assert _run(phases, flags) == 0
    want, base = [0] * 256, 0
    for p, n in enumerate([0, 3, 64, 1, 70, 5, 0, 40, 33]):
        want[base:base + n] = [11 + p] * n
        base += n
    assert flags.tolist() == want


def test_epoch_counter_and_wrap():
    """epoch + *epoch_dev at run time (graph replays), compared wrap-aware."""
    flags = torch.zeros(4, dtype=torch.int32, device=DEV)
    ctr = torch.zeros(1, dtype=torch.int32, device=DEV)
    assert L.lib().hiccl_counter_add(ctypes.c_void_p(ctr.data_ptr()), 5, _stream()) == 0
    assert _run([([0, 1], [0, 1], 1)], flags, epoch_dev=ctr) == 0
    assert flags[:2].tolist() == [6, 6]
    # 0xFFFFFFF0 + 0x20 wraps to 0x10: a flag holding 0x10 satisfies a wait
    # for 0x0000000F..0x10 and the wrapped epoch compares as newer
    flags.zero_()
    assert _run([([2], [2], 0xFFFFFFF0)], flags) == 0
    assert _run([([2], [2], 0x10)], flags) == 0
    assert flags[2].item() == 0x10


def test_timeout_sets_err_instead_of_hanging():
    flags = torch.zeros(4, dtype=torch.int32, device=DEV)
    assert _run([([0], [1], 3)], flags, timeout_s=0.05) == 1
    assert flags[0].item() == 3
    # a later phase still runs (err makes the remaining waits give up)
    assert _run([([], [1], 3), ([2], [], 4)], flags, timeout_s=0.05) == 1
    assert flags[2].item() == 4


def test_refuses_null_flags():
    arr = (Phase * 1)(Phase(None, 1, None, 0, 1))
    rc = L.lib().hiccl_signal_wait_phases(arr, 1, None, None, ctypes.c_double(1.0), _stream())
    assert rc != 0 and "signal" in L.last_error()
