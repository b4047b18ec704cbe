"""Deployment plumbing: K8s templates render to valid YAML, the container entrypoint builds the
right harness command, and the collective sweep runs (gloo, 2 ranks, CPU)."""
import glob
import json
import os
import re
import subprocess
import sys

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_k8s_templates_render():
    files = sorted(glob.glob(os.path.join(ROOT, "k8s", "*.yaml")))
    assert len(files) >= 7
    for f in files:
        text = re.sub(r"\{\{([A-Z_]+)\}\}", lambda m: "8" if m.group(1) in ("GPUS", "NNODES", "WORKERS") else "x",
                      open(f).read()).replace("__GPUS__", "1").replace("__IMAGE__", "img")
        docs = [d for d in yaml.safe_load_all(text) if d]
        assert docs, f
        for d in docs:
            assert "kind" in d and "metadata" in d


def _fake_python(tmp_path):
    bindir = tmp_path / "bin"
    bindir.mkdir()
    fake = bindir / "python3"
    fake.write_text("#!/bin/sh\necho ARGS: \"$@\"\n")
    fake.chmod(0o755)
    return str(bindir)


@pytest.mark.parametrize("gpus,strategy", [(1, "zero2"), (8, "fsdp")])
def test_entrypoint_command(tmp_path, gpus, strategy):
    env = dict(os.environ, PATH=_fake_python(tmp_path) + ":" + os.environ["PATH"], STRATEGY=strategy,
               NPROC_PER_NODE=str(gpus), APP=ROOT, STEPS="7", GRAD_ACCUM="4")
    out = subprocess.run(["bash", os.path.join(ROOT, "docker", "entrypoint.sh")], env=env, capture_output=True,
                         text=True, timeout=60).stdout
    line = [l for l in out.splitlines() if l.startswith("ARGS:")][0]
    assert "train_harness.py" in line and f"--strategy {strategy}" in line and "--steps 7" in line
    if gpus > 1:
        assert "torch.distributed.run" in line and f"--nproc-per-node {gpus}" in line
        assert "--fsdp-config" in line
    else:
        assert "--world-size 1" in line and "--deepspeed-config" in line


def test_collective_sweep_gloo(tmp_path):
    out = tmp_path / "c.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29561", os.path.join(ROOT, "scripts", "bench_collectives.py"),
           "--backend", "gloo", "--device", "cpu", "--dtype", "fp32", "--min-mb", "0.25", "--max-mb", "0.5",
           "--iters", "2", "--warmup", "1", "--ops", "all_reduce,reduce_scatter,all_gather", "--json", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    rows = json.loads(out.read_text())
    assert {x["op"] for x in rows} == {"all_reduce", "reduce_scatter", "all_gather"}
    assert all(x["busbw_GBps"] > 0 for x in rows)


def test_verify_offline_local():
    """scripts/verify_offline.sh (reference R38) in --local mode: imports, extension code object,
    model instantiation with the expected parameter counts, dataset, one CPU step."""
    import subprocess
    from dltb.ops._ext import so_path
    env = dict(os.environ, VERIFY_ALLOW_NO_EXT="0" if so_path() else "1")
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "verify_offline.sh"), "--local"],
                       capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "OFFLINE VERIFICATION PASSED" in r.stdout
    assert "TinyGPT tier A: 236.41M params" in r.stdout


def _fake_kubectl(tmp_path, plugin_pods):
    """A kubectl stand-in for scripts/check_cluster_gpus.sh (no cluster in the test container)."""
    bindir = tmp_path / "bin"
    bindir.mkdir()
    k = bindir / "kubectl"
    k.write_text(f"""#!/usr/bin/env bash
case "$*" in
  "cluster-info") echo ok ;;
  "config current-context") echo test-ctx ;;
  *"-l name=amdgpu-dp-ds"*) for i in $(seq 1 {plugin_pods}); do echo pod/amdgpu-dp-ds-$i; done ;;
  "get pods -A -o name") echo pod/coredns ;;
  "describe nodes") printf 'Name: mi355x-0\\n  amd.com/gpu: 8\\n' ;;
  *) exit 0 ;;
esac
""")
    k.chmod(0o755)
    return dict(os.environ, PATH=f"{bindir}:{os.environ['PATH']}")


@pytest.mark.parametrize("plugin_pods,ok", [(2, True), (0, False)])
def test_check_cluster_gpus(tmp_path, plugin_pods, ok):
    env = _fake_kubectl(tmp_path, plugin_pods)
    r = subprocess.run(["bash", os.path.join(ROOT, "scripts", "check_cluster_gpus.sh")], env=env,
                       capture_output=True, text=True, timeout=60)
    assert (r.returncode == 0) == ok, r.stdout + r.stderr
    assert ("CLUSTER READY" in r.stdout) == ok


def test_debug_extension_is_separate_and_loadable():
    """csrc/build.py --debug writes build/debug/_C*.so (never the release module) and DLTB_EXT_PATH
    loads it in place of the in-tree extension."""
    sys.path.insert(0, os.path.join(ROOT, "csrc"))
    try:
        import build as b
    finally:
        sys.path.pop(0)
    assert b.ext_path(True) != b.ext_path(False)
    assert os.path.dirname(b.ext_path(False)).endswith("distributed-llm-training-benchmark-framework_amd")
    dbg = b.ext_path(True)
    if not os.path.exists(dbg):
        pytest.skip("checked extension not built here (python csrc/build.py --debug)")
    r = subprocess.run([sys.executable, "-c", "import dltb; from dltb.ops._ext import so_path; print(so_path())"],
                       cwd=ROOT, env=dict(os.environ, DLTB_EXT_PATH=dbg), capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    assert r.stdout.strip().endswith(os.path.relpath(dbg, ROOT).split(os.sep, 1)[1]) or dbg in r.stdout
