"""Bit-for-bit comparison of two builds of libswarm_hip.so on the same training ticks.

Each library runs in its own child process (SWARM_LIB_PATH; "base" = the in-tree library): a fused
engine of the given configuration is prefilled with acting ticks, then runs `ticks` training ticks;
the gradient after every tick and the final weights, Adam moments, target and control block are
saved.  The parent reports whether the two runs agree bit for bit (a kernel change meant to move
only stores or schedules must leave every bit alone).

usage: python tools/bitcmp.py LIB_A LIB_B [scenario N B ticks]   (LIB = base or a path)
"""
import json
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, numpy as np, torch
sys.path.insert(0, %(root)r)
import swarm_amd
scen, N, B, T, out = %(scen)r, %(N)d, %(B)d, %(T)d, %(out)r
key = "weights_go_to" if scen == "GoTo" else "weights_obstacle_avoidance"
w0 = torch.tensor(np.load(os.path.join(%(root)r, "tests", "golden", "weights.npz"))[key][0])
eng = swarm_amd.SwarmEngine(scen, N, B, seed=3, params=w0, batch=B, eps=0.2, replay_capacity=8 * B,
                            update_target_every=3)
eng.reset(0)
for _ in range(3):
    eng.act(push=True, full_out=False)
    eng.advance()
grads = []
for t in range(T):
    eng.train_tick()
    torch.cuda.synchronize()
    grads.append(eng.grad.cpu().clone())
eng.flush()
torch.cuda.synchronize()
torch.save({"grads": torch.stack(grads), "params": eng.params.cpu(), "m": eng.adam_m.cpu(), "v": eng.adam_v.cpu(),
            "target": eng.target.cpu(), "ctrl": eng.ctrl.cpu(), "ho": eng.handoff_errors(),
            "build": swarm_amd._lib.load().swarm_build_info().decode()}, out)
"""


def run(lib, scen, N, B, T, out):
    env = dict(os.environ)
    if lib != "base":
        env["SWARM_LIB_PATH"] = os.path.abspath(lib)
    else:
        env.pop("SWARM_LIB_PATH", None)
    code = CHILD % dict(root=ROOT, scen=scen, N=N, B=B, T=T, out=out)
    subprocess.run([sys.executable, "-c", code], env=env, check=True, timeout=300)


def main():
    import torch
    a, b = sys.argv[1], sys.argv[2]
    scen = sys.argv[3] if len(sys.argv) > 3 else "GoTo"
    N = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    B = int(sys.argv[5]) if len(sys.argv) > 5 else 1024
    T = int(sys.argv[6]) if len(sys.argv) > 6 else 6
    with tempfile.TemporaryDirectory() as d:
        pa, pb = os.path.join(d, "a.pt"), os.path.join(d, "b.pt")
        run(a, scen, N, B, T, pa)
        run(b, scen, N, B, T, pb)
        ra, rb = torch.load(pa, weights_only=True), torch.load(pb, weights_only=True)
    res = {"a": a, "b": b, "build_a": ra["build"], "build_b": rb["build"], "config": [scen, N, B, T],
           "handoff_errors": [ra["ho"], rb["ho"]]}
    for k in ("grads", "params", "m", "v", "target", "ctrl"):
        res[k + "_bitwise"] = bool(torch.equal(ra[k], rb[k]))
    res["grad_max_abs_diff"] = float((ra["grads"] - rb["grads"]).abs().max())
    res["all_bitwise"] = all(res[k + "_bitwise"] for k in ("grads", "params", "m", "v", "target", "ctrl"))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
