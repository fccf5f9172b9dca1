"""The driver's one JSON line from bench.py's full record: every contract
field, the roofline, CPU-baseline and config-5 summaries, a few KB at any
N (the driver keeps a tail of stdout); the full record goes to stderr
("bench-detail").  Pure functions, no GPU."""


def compact_line(line):
    """The driver's line: every contract field, the roofline and CPU-baseline
    summaries and the config-5 verdicts, without the per-pass lists and
    per-mode host splits the full record (stderr, "bench-detail") carries --
    a few KB at any N, so the driver's stdout tail always holds all of it."""
    out = dict(line)
    r = dict(line["roofline"])
    srw = r.pop("serial_rw_model", None) or {}
    r["serial_rw_frac"] = srw.get("frac_write_probe")
    r["serial_rw_frac_copy_write"] = srw.get("frac")
    tp = r.pop("traffic_from_profile", None) or {}
    # the cited profile, its kernel time and whether that time fits this run's
    # kernel mean (a profile from a slower box does not)
    r["traffic_profile"] = ({"file": tp.get("file"), "kernel_ms": tp.get("box_kernel_ms"),
                             "fits_this_run": tp.get("fits_this_run"), "x_alg": tp.get("over_algorithmic")}
                            if tp else None)
    r.pop("traffic_source", None)
    out["roofline"] = r
    cpu = line.get("cpu_baseline")
    if cpu:
        c = {k: cpu.get(k) for k in ("value", "unit", "cores", "kind", "min", "max", "max_over_min", "passes")}
        c["sample"] = cpu.get("sample", "")[:200]
        pl = cpu.get("placement") or {}
        c["placement"] = {"policy": pl.get("policy"), "numa_nodes": pl.get("numa_nodes"), "l3_domains": pl.get("l3_domains")}
        th = cpu.get("throttle")
        c["throttled_ms"] = round(th.get("throttled_usec", 0) * 1e-3, 1) if th else None
        sc = cpu.get("spread_cause")
        if isinstance(sc, str):
            c["spread_cause"] = {"cause": sc}
        elif sc:
            c["spread_cause"] = {k: sc.get(k) for k in ("cause", "slow_passes", "slow_runs", "throttle_covers_frac",
                                                         "pages_local", "host_busy_others_median")}
        out["cpu_baseline"] = c
    pf = line.get("parity_full")
    if pf:
        out["parity_full"] = {k: pf.get(k) for k in ("ok", "mismatches", "words")}
    dp = line.get("device_props") or {}
    out["device_props"] = {k: dp.get(k) for k in ("gcn_arch", "cus", "peak_GBps_from_props_x4")}
    mis = line.get("c2_misaligned")
    if mis:
        out["c2_misaligned"] = {"shifted_over_aligned": mis.get("shifted_over_aligned"),
                                "shifted_over_headline": mis.get("shifted_over_headline"),
                                "aligned_over_headline": mis.get("aligned_over_headline"),
                                "shifted_frac": mis.get("shifted_frac"),
                                "parity_ok": all((mis.get("parity_sample_ok") or {"": False}).values())}
    lab = line.get("c2_layout_ab")
    if lab:
        out["c2_layout_ab"] = {k: lab.get(k) for k in ("separate_over_bucket", "separate_over_headline", "bucket_frac",
                                                       "separate_frac", "outputs_identical")}
    if line.get("c5") is not None:
        out["c5"] = compact_c5(line["c5"])
    return out


def compact_c5(c5):
    """Per config-5 mode: its known-answer verdict, exit code, median
    collective time and rate, step-kernel time and the mode that ran."""
    out = {k: c5[k] for k in ("skipped", "stopped_after", "forced_stream_ordered") if k in c5}
    if "workload" in c5:
        out["workload"] = str(c5["workload"])[:120]
    for name, r in c5.items():
        if not isinstance(r, dict) or name in ("env_scrubbed", "protocol_ab"):
            continue
        m = {"kat": r.get("kat"), "rc": r.get("rc"), "ms": r.get("collective_ms_median"),
             "GBps": r.get("algorithmic_GBps_median"), "kernel_us_step": r.get("kernel_us_per_step_rank0"),
             "mode_used": r.get("mode_used")}
        for k in ("skipped", "error"):  # the head of the message names the failure
            if k in r:
                m[k] = str(r[k])[:100]
        out[name] = {k: v for k, v in m.items() if v is not None}
    ab = c5.get("protocol_ab")
    if ab:
        out["protocol_ab"] = {"baseline_ms": ab.get("baseline_ms"),
                              **{k: (v or {}).get("over_baseline") for k, v in ab.items() if isinstance(v, dict)}}
    return out
