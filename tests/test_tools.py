"""CPU tier: the GPU-call wrapper keeps a failed attempt's logs.

tools/gpurun_call.sh runs one gpurun call and logs it; after an attempt
whose status is not ok it renames every gpurun_out/ entry of the tag that the
attempt pulled back to TAG_aN_*, so a retry into the same file names cannot
overwrite the failure.  Checked here with a stub client
(HICCL_GPURUN) in a scratch tree: no GPU, no gpurun.
"""
import os
import shutil
import stat
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "tools", "gpurun_call.sh")

STUB = """#!/usr/bin/env bash
# stub gpurun: runs the command locally, then prints gpurun's status line
# (fail while FAIL_FILE exists)
shift 3  # --timeout N --
bash -c "$1"
if [ -e "$FAIL_FILE" ]; then echo "[gpurun] status=fail rc=1 charged=1.0s"; exit 1; fi
echo "[gpurun] status=ok rc=0 charged=1.0s"
"""


def _setup(tmp_path):
    (tmp_path / "tools").mkdir()
    shutil.copy(SCRIPT, tmp_path / "tools" / "gpurun_call.sh")
    stub = tmp_path / "stub_gpurun"
    stub.write_text(STUB)
    stub.chmod(stub.stat().st_mode | stat.S_IEXEC)
    (tmp_path / "gpurun_out").mkdir()
    (tmp_path / "gpurun_out" / "r99x_bench.jsonl").write_text("an older run's result\n")  # not pulled: kept
    return stub


def _call(tmp_path, stub, tag, cmd, fail):
    env = dict(os.environ, HICCL_GPURUN=str(stub), FAIL_FILE=str(tmp_path / "FAIL"))
    if fail:
        (tmp_path / "FAIL").write_text("")
    elif (tmp_path / "FAIL").exists():
        (tmp_path / "FAIL").unlink()
    return subprocess.run(["bash", str(tmp_path / "tools" / "gpurun_call.sh"), tag, "60", cmd], env=env,
                          capture_output=True, text=True, timeout=60)


def test_failed_attempt_logs_survive_the_retry(tmp_path):
    stub = _setup(tmp_path)
    out = tmp_path / "gpurun_out"
    cmd = 'echo "suite output of attempt $(date +%N)" > gpurun_out/r99x_gputest.log; mkdir -p gpurun_out/prof_r99x; ' \
          'echo trace > gpurun_out/prof_r99x/stats.csv'
    r1 = _call(tmp_path, stub, "r99x", cmd.replace("attempt", "FAILING attempt"), fail=True)
    assert r1.returncode == 1
    r2 = _call(tmp_path, stub, "r99x", cmd, fail=False)
    assert r2.returncode == 0
    names = sorted(os.listdir(out))
    # attempt 1's pulled entries kept under attempt-suffixed names, the retry's under the plain ones
    assert "FAILING" in (out / "r99x_a1_gputest.log").read_text()
    assert "FAILING" not in (out / "r99x_gputest.log").read_text()
    assert (out / "r99x_a1_prof_r99x" / "stats.csv").exists() and (out / "prof_r99x" / "stats.csv").exists()
    # an entry the failed attempt did not touch stays where it was
    assert (out / "r99x_bench.jsonl").read_text() == "an older run's result\n"
    assert "r99x_a1_bench.jsonl" not in names
    att = (out / "r99x_attempts.log").read_text().splitlines()
    assert [ln.split()[2] for ln in att if " gpurun_rc " in ln] == ["1", "2"]
    assert "status=fail" in att[0] and "kept 2 pulled entries as r99x_a1_*" in att[1] and "status=ok" in att[2]
    # the call log holds both attempts' client output
    assert (out / "r99x_call.log").read_text().count("[gpurun] status=") == 2


def test_second_failure_gets_its_own_suffix(tmp_path):
    stub = _setup(tmp_path)
    out = tmp_path / "gpurun_out"
    for k in (1, 2):
        _call(tmp_path, stub, "r99y", f'echo fail{k} > gpurun_out/r99y_gputest.log', fail=True)
    assert (out / "r99y_a1_gputest.log").read_text() == "fail1\n"
    assert (out / "r99y_a2_gputest.log").read_text() == "fail2\n"
    assert not (out / "r99y_gputest.log").exists()


def test_archive_stays_off_the_gpu_box():
    """tools/archive/ (retired probes; their results live in profiles/) is
    not pushed to the GPU box, and nothing the GPU tier, smoke() or bench.py
    runs imports from it."""
    import re
    ignore = open(os.path.join(ROOT, ".gpurunignore")).read().split()
    assert "./tools/archive" in ignore
    users = [os.path.join(ROOT, f) for f in ("bench.py", "__graft_entry__.py")]
    users += [os.path.join(ROOT, "tools", f) for f in os.listdir(os.path.join(ROOT, "tools")) if f.endswith(".py")]
    users += [os.path.join(ROOT, "tests", f) for f in os.listdir(os.path.join(ROOT, "tests")) if f.endswith(".py")]
    pat = re.compile(r"^\s*(import|from)\s+\S*archive|sys\.path\.\w+\(.*archive", re.M)
    for f in users:
        assert not pat.search(open(f).read()), f
