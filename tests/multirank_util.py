"""Shared driver + comparison for the world-size equivalence tests (scripts/multirank_check.py)."""
import os
import socket
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCRIPT = os.path.join(ROOT, "scripts", "multirank_check.py")


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run(out, world, device, extra=(), env_extra=None, timeout=900):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    if world == 1:
        cmd = [sys.executable, SCRIPT]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", "--max-restarts=0", SCRIPT]
    r = subprocess.run(cmd + ["--out", str(out), "--device", device, *extra], capture_output=True,
                       text=True, env=env, timeout=timeout)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-5000:])
    return torch.load(str(out), weights_only=True)


def compare(ref, got, loss_tol, upd_tol, cos_min, param_tol):
    """Per case: identical init, loss curves within ``loss_tol`` (relative), parameter updates
    (final - init over all parameters) within ``upd_tol`` relative L2 and cosine >= ``cos_min``,
    and every parameter whose update is >= 5 % of the largest one within ``param_tol``."""
    bad = []
    for case, r in ref.items():
        g = got[case]
        for n in r["init"]:
            assert torch.equal(r["init"][n], g["init"][n]), (case, n, "init differs")
        for a, b in zip(r["losses"], g["losses"]):
            if abs(a - b) > loss_tol * abs(a):
                bad.append((case, "loss", a, b))
                break
        ur = {n: r["final"][n] - r["init"][n] for n in r["init"]}
        ug = {n: g["final"][n] - g["init"][n] for n in r["init"]}
        vr = torch.cat([ur[n].reshape(-1) for n in ur]).double()
        vg = torch.cat([ug[n].reshape(-1) for n in ur]).double()
        rel = ((vg - vr).norm() / vr.norm()).item()
        cos = (torch.dot(vg, vr) / (vg.norm() * vr.norm())).item()
        if rel > upd_tol or cos < cos_min:
            bad.append((case, "update", rel, cos))
        top = max(ur[n].norm().item() for n in ur)
        for n in ur:
            nr = ur[n].norm().item()
            if nr >= 0.05 * top:
                pr = ((ug[n] - ur[n]).norm() / nr).item()
                if pr > param_tol:
                    bad.append((case, n, pr))
    return bad


def report(ref, got):
    """Per case: max relative loss gap, update rel-L2 / cosine and the largest per-parameter update
    gap (the quantities ``compare`` bounds), for recording how tight a run actually is."""
    out = {}
    for case, r in ref.items():
        g = got[case]
        ur = {n: r["final"][n] - r["init"][n] for n in r["init"]}
        ug = {n: g["final"][n] - g["init"][n] for n in r["init"]}
        vr = torch.cat([ur[n].reshape(-1) for n in ur]).double()
        vg = torch.cat([ug[n].reshape(-1) for n in ur]).double()
        top = max(ur[n].norm().item() for n in ur)
        prel = max(((ug[n] - ur[n]).norm() / ur[n].norm()).item() for n in ur if ur[n].norm().item() >= 0.05 * top)
        out[case] = {"loss_rel": max(abs(a - b) / abs(a) for a, b in zip(r["losses"], g["losses"])),
                     "upd_rel": ((vg - vr).norm() / vr.norm()).item(),
                     "upd_cos": (torch.dot(vg, vr) / (vg.norm() * vr.norm())).item(),
                     "param_rel_max": prel}
    return out
