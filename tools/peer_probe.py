"""Diagnostic: do two in-process streams run their peer all-reduce launches side by side?

The single-process emulation of W ranks (tests/test_gpu_peer.py) needs every rank's kernels
to be co-resident with the others' (they wait on each other's stores).  This launches a W = 2
swarm_peer_allreduce on stream pairs made several ways and reports, per trial, the expired
waits of each rank (short bound, 20 ms).  Prints one JSON line per mode."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import swarm_amd  # noqa: E402
from swarm_amd.dist import PeerExchange  # noqa: E402


def trial(ends, ss, x):
    before = [e.errors() for e in ends]
    for r, s in enumerate(ss):
        with torch.cuda.stream(s):
            ends[r].allreduce_(x[r])
    torch.cuda.synchronize()
    return [e.errors() - b for e, b in zip(ends, before)]


def main():
    swarm_amd.load_library()
    ends = PeerExchange.local(2, timeout_us=20000)
    x = [torch.ones(1674, device="cuda") for _ in range(2)]
    modes = {
        "fresh pool streams per trial": lambda: [torch.cuda.Stream() for _ in range(2)],
        "fresh high-priority pool streams": lambda: [torch.cuda.Stream(priority=-1) for _ in range(2)],
    }
    fixed = [torch.cuda.Stream() for _ in range(2)]
    modes["one fixed pair"] = lambda: fixed
    for name, mk in modes.items():
        res = []
        for _ in range(24):
            ss = mk()
            res.append(trial(ends, ss, x) + [hex(ss[0].cuda_stream)[-5:], hex(ss[1].cuda_stream)[-5:]])
        bad = sum(1 for r in res if r[0] or r[1])
        print(json.dumps({"mode": name, "bad_trials": bad, "trials": res}))
    ends[0].close()


if __name__ == "__main__":
    main()
