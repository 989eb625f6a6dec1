"""GPU: the halo exchange on real RCCL (torch.distributed "nccl").

A one-GPU box cannot hold two RCCL ranks ("Duplicate GPU detected",
tools/probe_rccl_one_gpu.py), so tests/rccl_loopback.py runs a one-rank RCCL
group in a child process with a loopback plan: every source row the
aggregation reads comes through an RCCL collective (dense all-gather or
sparse all-to-all-v), in HaloPipeline's side-stream / async branch and in
_HaloExchange's synchronous one; the row-pipelined one-kernel layer, whose
backward posts the halo block's partials point to point (batch_isend_irecv);
and the bucketed gradient all-reduce.  The child prints its checks as JSON."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def test_halo_exchange_on_rccl_loopback():
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "rccl_loopback.py")], env=env,
                       capture_output=True, text=True, timeout=240)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"rc {r.returncode}\nstdout:\n{r.stdout[-3000:]}\nstderr:\n{r.stderr[-3000:]}"
    res = json.loads(lines[-1])
    failed = {k: v for k, v in res["checks"].items() if not (v is True or (isinstance(v, dict) and v["ok"]))}
    assert not failed and res["ok"] and r.returncode == 0, (failed, r.stderr[-2000:])
    assert res["backend"] == "nccl"
    assert res["dense_halo_rows"] > 0 and res["sparse_halo_rows"] > 0
    # the row-pipelined backward had a halo block to post point to point (the loopback peer's rows)
    assert res["dense_rows_blocks"] and res["dense_rows_blocks"][0][1] > 0
    assert res["sparse_rows_blocks"] and res["sparse_rows_blocks"][0][1] > 0


def test_sharded_model_on_rccl_loopback():
    """tests/loopback_model.py: the drop-in model's training step and streamed
    inference over a loopback shard with every grl.dist collective on a
    one-rank RCCL group -- bitwise the same steps over a one-rank LocalGroup
    (the emulator the multi-rank GPU tests run), the forward bitwise the
    one-GPU model's -- and each kind of collective actually issued to RCCL."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, "-u", os.path.join(HERE, "loopback_model.py")], env=env,
                       capture_output=True, text=True, timeout=400)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert lines, f"rc {r.returncode}\nstdout:\n{r.stdout[-3000:]}\nstderr:\n{r.stderr[-3000:]}"
    res = json.loads(lines[-1])
    failed = {k: v for k, v in res["checks"].items() if not (v is True or (isinstance(v, dict) and v["ok"]))}
    assert not failed and res["ok"] and r.returncode == 0, (failed, res["calls"], r.stderr[-2000:])
    assert res["backend"] == "nccl"
