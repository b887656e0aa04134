"""The C4 exchange watchdog of bench.py (CPU, gloo, world size 2): a rank
stuck in a collective ends the run with EXIT_EXCHANGE_FAILED after rank 0
prints its line marked unverified; an exchange that completes first is never
cut short and prints nothing twice."""
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

_RANK = r"""
import json, os, sys, time
sys.path.insert(0, os.environ["ROOT"])
import bench, torch, torch.distributed as dist
r, mode = int(os.environ["RANK"]), os.environ["MODE"]
dist.init_process_group("gloo", rank=r, world_size=2, init_method="tcp://127.0.0.1:" + os.environ["PORT"])
def on_timeout():
    if r == 0:
        print(json.dumps({"c4_exchange": {"error": "no result", "verified": False}}), flush=True)
    return bench.EXIT_EXCHANGE_FAILED
g = bench.ExchangeGuard(float(os.environ["TMO"]), on_timeout).start()
if mode == "hang" and r == 1:
    time.sleep(120)
t = torch.ones(1)
dist.all_reduce(t)
g.finish()
time.sleep(float(os.environ["TMO"]) + 1.0)  # past the timeout: a late timer must stay silent
print("finished", int(t.item()), flush=True)
dist.destroy_process_group()
"""


def _port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(mode: str, tmo: float):
    port = str(_port())
    procs = []
    for r in range(2):
        env = dict(os.environ, ROOT=ROOT, RANK=str(r), MODE=mode, PORT=port, TMO=str(tmo), MASTER_ADDR="127.0.0.1")
        procs.append(subprocess.Popen([sys.executable, "-c", _RANK], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        try:
            o, e = p.communicate(timeout=90)
        except subprocess.TimeoutExpired:
            p.kill()
            o, e = p.communicate()
        outs.append((p.returncode, o, e))
    return outs


def test_exchange_hang_exits_nonzero_with_line():
    import bench

    outs = _run("hang", 3.0)
    assert [rc for rc, _, _ in outs] == [bench.EXIT_EXCHANGE_FAILED] * 2, outs
    lines = [ln for ln in outs[0][1].splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and '"verified": false' in lines[0], outs[0]
    assert "finished" not in outs[0][1] and "finished" not in outs[1][1]


def test_exchange_done_first_is_never_cut():
    outs = _run("ok", 2.0)
    for rc, o, e in outs:
        assert rc == 0, (rc, o, e)
        assert o.count("finished 2") == 1 and "{" not in o, o
