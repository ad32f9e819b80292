"""bench.py's multi-rank launch (VERDICT r3 "next" #1), on the CPU: no GPU is touched.

``python bench.py --gpus N`` with no launcher (WORLD_SIZE unset) must start its own N ranks as a
child ``torch.distributed.run`` before any GPU call, relay rank 0's JSON line and exit non-zero
when a rank fails or the line does not report N GPUs; under a launcher, WORLD_SIZE must equal N.
The spawn path is exercised end to end with stand-in rank scripts.
"""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (module import only: bench.main() is not called)


def test_launch_decision():
    assert bench.launch_decision(1, {}) == "run"
    assert bench.launch_decision(8, {}) == "spawn"
    assert bench.launch_decision(2, {"WORLD_SIZE": "2"}) == "run"
    assert bench.launch_decision(1, {"WORLD_SIZE": "1"}) == "run"
    with pytest.raises(SystemExit):
        bench.launch_decision(8, {"WORLD_SIZE": "1"})
    with pytest.raises(SystemExit):
        bench.launch_decision(1, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.launch_decision(0, {})


def test_rank_launch_command():
    cmd = bench.rank_launch_cmd(["--gpus", "4", "--steps", "3"], 4, 29512)
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29512" in cmd
    assert cmd[-5:] == [os.path.join(ROOT, "bench.py"), "--gpus", "4", "--steps", "3"]


RANK_SCRIPT = """
import json, os, sys
rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
mode = sys.argv[1]
if mode == "fail" and rank == 1:
    sys.exit(7)
if rank == 0:
    print("progress text")
    print(json.dumps({"metric": "m", "n_gpus": 1 if mode == "short" else world, "args": sys.argv[1:]}))
"""


@pytest.mark.parametrize("mode,want", [("ok", 0), ("short", 3), ("fail", "nonzero")])
def test_spawn_ranks_relays_and_checks(tmp_path, capsys, mode, want):
    script = tmp_path / "rank.py"
    script.write_text(RANK_SCRIPT)
    rc = bench.spawn_ranks([mode], 2, script=str(script))
    out = capsys.readouterr().out
    if want == "nonzero":
        assert rc != 0
        return
    assert rc == want
    lines = [json.loads(x) for x in out.splitlines() if x.startswith("{")]
    assert len(lines) == 1 and lines[0]["args"] == [mode]   # rank 0's line, relayed once
    assert "progress text" in out


HANG_SCRIPT = """
import os, sys, time
with open(os.path.join(sys.argv[1], "pid%s" % os.environ["RANK"]), "w") as f:
    f.write(str(os.getpid()))
time.sleep(600)
"""

RELAY = """
import sys
sys.path.insert(0, %r)
import bench
sys.exit(bench.spawn_ranks([%r], 2, script=%r))
"""


def test_sigterm_to_the_relay_stops_the_ranks(tmp_path):
    """the rank launcher runs in its own session, so a SIGTERM to the relaying bench.py
    (timeout(1), a harness) must still end the ranks: the relay's handler turns it into
    SystemExit and its finally block terminates the launcher's process group."""
    import signal
    import subprocess
    import time
    script = tmp_path / "hang.py"
    script.write_text(HANG_SCRIPT)
    relay = subprocess.Popen([sys.executable, "-c", RELAY % (ROOT, str(tmp_path), str(script))])
    pids = []
    t0 = time.time()
    while len(pids) < 2 and time.time() - t0 < 120:
        pids = [int((tmp_path / f"pid{r}").read_text()) for r in range(2) if (tmp_path / f"pid{r}").exists()
                and (tmp_path / f"pid{r}").read_text()]
        time.sleep(0.2)
    assert len(pids) == 2, "ranks did not start"
    relay.send_signal(signal.SIGTERM)
    assert relay.wait(timeout=60) != 0
    deadline = time.time() + 30
    alive = pids
    while alive and time.time() < deadline:
        alive = []
        for p in pids:
            try:
                os.kill(p, 0)
                alive.append(p)
            except ProcessLookupError:
                pass
        time.sleep(0.2)
    for p in alive:   # clean up before failing
        os.kill(p, signal.SIGKILL)
    assert not alive, f"ranks {alive} outlived the relay"
