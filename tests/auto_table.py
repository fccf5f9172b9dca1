"""AUTO's expected choices, ONE table for both tiers.

The CPU tier (tests/test_abi.py) checks every row against
hiccl_reduce_auto_choice(_ex) on the host; the GPU tier
(tests/test_reduce_gpu.py) runs the same rows on the device and checks the
engine / store form the plan actually took against the row AND against the
host answer for the device's CU count.  A change of AUTO's rule that is not
carried into this table fails the CPU tier first, before any GPU minute is
spent (the GPU tier kept its own copy of the rule and
went red after two rule changes).

Rule: DESIGN.md section 4 (AUTO table, store form by launch size);
hiccl_amd/csrc/reduce.hip auto_engine / oneshot_cfg / plan_store_peer.
"""
import hiccl_amd._lib as L

T, P = L.HICCL_ENGINE_TILE, L.HICCL_ENGINE_PHASE
F32, BF16, F64, U64, I32, BYTES = (L.HICCL_FLOAT32, L.HICCL_BFLOAT16, L.HICCL_FLOAT64, L.HICCL_UINT64,
                                   L.HICCL_INT32, L.HICCL_BYTES)
MiB = 1 << 20
NT, WT = 2, 4  # hiccl_reduce_config_t.store_policy values

# (dtype, elements per input, n) -> (engine, unroll, blocks per CU, dynamic),
# 256 CUs, default config
RULE_CASES = [
    ((F32, 1 << 28, 8), (T, 4, 1, 1)),        # C2: tiles on the ticket counter
    ((F32, 1 << 26, 2), (T, 4, 1, 0)),        # C3, two inputs: static tiles
    ((F32, 1 << 26, 3), (T, 4, 1, 0)),        # C3, 3 inputs, write-through (round 5): static tiles
    ((F32, 1 << 26, 4), (P, 16, 1, 0)),       # C3, 4 inputs: 8 whole chunks per CU
    ((F32, 1 << 27, 3), (P, 16, 1, 0)),       # 512 MiB written (nt): the phased engine
    ((F32, 1 << 26, 8), (P, 16, 1, 0)),       # C3, many inputs, write-through (round 5): PHASE
    ((F32, 1 << 26, 64), (P, 16, 1, 0)),
    ((F32, 1 << 27, 8), (T, 4, 1, 1)),        # 512 MiB written (nt): 128 tickets per workgroup, tiles
    ((BF16, 1 << 27, 8), (P, 16, 1, 0)),      # bf16 256 MiB per input, write-through: PHASE too
    ((BF16, 1 << 28, 8), (T, 4, 1, 1)),       # bf16 512 MiB (nt): tiles
    ((F32, 1 << 28, 2), (T, 16, 1, 1)),       # 1 GiB per input, few inputs: wide tiles
    ((F32, 1 << 28, 3), (T, 8, 1, 1)),
    ((F32, 40 * MiB // 4, 3), (T, 4, 1, 0)),  # 1.25 chunks per CU: tiles
    ((F32, 32 * MiB // 4, 4), (T, 4, 1, 0)),  # one chunk per CU, 3-4 inputs: tiles
    ((F32, 40 * MiB // 4, 8), (T, 4, 1, 0)),  # a last round 25 % busy: tiles
    ((F32, 48 * MiB // 4, 8), (P, 16, 1, 0)),  # 75 % busy: PHASE
    ((F32, 24 * MiB // 4, 16), (P, 16, 1, 0)),  # 16 inputs, 0.75 chunks per CU: PHASE
    ((F32, 16 * MiB // 4, 16), (T, 4, 4, 0)),   # 0.5 per CU: tiles, 4 workgroups per CU
    ((F32, 5 << 18, 2.4), (T, 2, 4, 0)),      # the C5 step's plan: half-size tiles
    ((BF16, 40 * MiB // 2, 3), (T, 4, 1, 0)),  # bf16 native: the f32 rule
    ((F64, 40 * MiB // 8, 3), (T, 4, 1, 0)),   # f64 / u64 too (r03x_midsize_f64.jsonl)
    ((F64, (1 << 26) // 2, 3), (P, 16, 1, 0)),
    ((U64, 40 * MiB // 8, 8), (T, 4, 1, 0)),
]

# The GPU tier's plan cases (one compute each): (dtype, elements per input,
# n, config) -> engine.  test_plan_auto_engine_picks_phase_for_large_buckets
# (f32), test_plan_auto_engine_bf16, test_auto_wide_tiles_large_few_inputs.
_C = 1 << 23
GPU_PLAN_ENGINE_F32 = [
    ((F32, 1 << 27, 6, None), T),   # 512 MiB written (nt), >= 64 tickets per workgroup: tiles
    ((F32, 1 << 26, 6, None), P),   # write-through, many inputs: PHASE
    ((F32, _C, 6, None), P),
    ((F32, _C, 2, None), T),
    ((F32, 1 << 24, 2, None), T),
    ((F32, 1 << 26, 4, None), P),
    ((F32, _C // 4, 6, None), T),
    ((F32, _C // 4, 2, None), T),
    ((F32, _C, 4, None), T),
    ((F32, _C * 5 // 4, 8, None), T),   # 1.25 chunks per CU: tiles
    ((F32, _C * 3 // 2, 8, None), P),
    ((F32, _C * 9 // 2, 3, None), T),   # three f32 inputs, write-through: static tiles
    ((F32, _C * 5 // 2, 4, None), T),
    ((F32, _C * 9 // 2, 3, dict(store_policy=NT)), P),  # the same with nt stores asked for: the nt table
]
GPU_PLAN_ENGINE_BF16 = [  # 8 mutually misaligned inputs
    ((BF16, 1 << 28, 8, None), T),  # 512 MiB written (nt): tiles
    ((BF16, 1 << 27, 8, None), P),  # 256 MiB (write-through): PHASE
    ((BF16, 1 << 26, 8, None), P),
]
GPU_WIDE_TILES = [((dt, (1 << 30) // esz, n, None), T) for dt, esz in ((F32, 4), (BF16, 2)) for n in (2, 3, 4)]

# Store forms the GPU tier checks on plans: (dtype, total elements written,
# packet-weighted mean n, config) -> store_policy.
STEP = 5 << 18  # the C5 step: 4 x n = 2 + 1 x n = 4 computes of 2^18 f32 (mean n 2.4)
GPU_STORE_SMALL_STEP = {  # test_plan_store_form_small_step ids
    "auto": ((F32, STEP, 2.4, None), WT),
    "nt": ((F32, STEP, 2.4, dict(store_policy=NT)), NT),
    "wt": ((F32, STEP, 2.4, dict(store_policy=WT)), WT),
    "phase": ((F32, STEP, 2.4, dict(engine=P)), WT),
    "u2": ((F32, STEP, 2.4, dict(engine=T, unroll=2)), WT),
    "u1-nt": ((F32, STEP, 2.4, dict(engine=T, unroll=1)), NT),
}
GPU_STORE_LARGE = {  # test_plan_store_form_large ids: 8 inputs in 1 MiB computes
    "64MiB-auto-wt": ((F32, 1 << 24, 8, None), WT),
    "512MiB-auto-nt": ((F32, 1 << 27, 8, None), NT),
    "512MiB-wt": ((F32, 1 << 27, 8, dict(store_policy=WT)), WT),
}
GPU_STORE_BYTES = [  # test_byte_copy_plan_store_forms
    ((BYTES, 48 << 20, 1, None), NT),
    ((BYTES, 5 * ((1 << 20) + 3), 1, None), WT),
]


def all_engine_rows():
    return GPU_PLAN_ENGINE_F32 + GPU_PLAN_ENGINE_BF16 + GPU_WIDE_TILES


def all_store_rows():
    return list(GPU_STORE_SMALL_STEP.values()) + list(GPU_STORE_LARGE.values()) + GPU_STORE_BYTES
