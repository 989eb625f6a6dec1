"""CPU: bench.py's launch handling for the driver's N > 1 runs.

  * under a launcher (WORLD_SIZE set) --gpus must equal WORLD_SIZE, else it
    exits non-zero before touching a GPU;
  * `--gpus N` without a launcher starts N rank processes itself; when a rank
    fails (here: no GPU in this container) the parent stops and exits
    non-zero instead of hanging or printing a one-GPU line.
The GPU half (two gloo ranks print one line with n_gpus 2) is
tests/test_gpu_dist.py::test_bench_spawns_its_ranks_without_a_launcher."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env_over):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_over)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=240)


def test_world_size_mismatch_is_an_error():
    r = _bench(["--gpus", "8", "--cpu-seconds", "0"], WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr and "--gpus 8" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_spawned_ranks_fail_loudly_without_a_gpu():
    r = _bench(["--gpus", "2", "--dist-backend", "gloo", "--cpu-seconds", "0"])
    assert r.returncode != 0
    assert "no ROCm GPU visible" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())


def test_gpus_must_be_positive():
    r = _bench(["--gpus", "0"])
    assert r.returncode != 0 and "--gpus must be >= 1" in r.stderr


def test_pmc_traffic_is_keyed_by_workload_world_and_kernel():
    """roofline.traffic comes only from a PMC record of the same workload, at
    the same world size and shard shape, on the same kernel family: the C3
    one-GPU record is found; C4's rank-0 shards at P = 2 / 4 / 8 find the
    records tools/pmc_rank_traffic.py wrote for their slice kernels (n_loc =
    1M at P = 4 is also C3's row count: the world size and kernel keep them
    apart); any other shard shape or kernel gets None (traffic: null)."""
    import argparse
    import importlib.util

    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    a = argparse.Namespace(graph="er", avg_deg=32.0, types=6, dim=256, p=0.0)
    one = "spmm_kernel<4,1,8,false,false> (grl_typed_spmm_fwd)"
    shard = "spmm_kernel / spmm_pair_kernel (grl_typed_spmm_fwd_slice, 2 slices of 128 columns)"
    assert bench.load_traffic(a, "C3", 1_000_000, 1, one) > 3e10
    c4 = {P: bench.load_traffic(a, "C4", 4_000_000 // P, P, shard) for P in (2, 4, 8)}
    assert 7e10 < c4[2] < 9e10 and 3.5e10 < c4[4] < 4.5e10 and 1.7e10 < c4[8] < 2.3e10, c4
    assert bench.load_traffic(a, "C4", 1_000_000, 4, one) is None  # the one-GPU kernel's string: not this record
    assert bench.load_traffic(a, "C4", 1_500_000, 2, shard) is None  # another shard shape
    assert bench.load_traffic(a, "C4", 1_000_000, 1, one) is None  # C4 has no one-GPU record
    assert bench.load_traffic(a, "C3", 1_000_000, 1, "gemm_x6_kernel") is None  # another kernel's bytes: never


def test_unknown_path_option_is_refused_before_any_work():
    """bench.py --option NAME=VALUE sets a libgrl path option (grl_set_option)
    for the run; an unknown name fails at once, naming it, with no JSON line."""
    r = _bench(["--option", "no_such_option=1", "--cpu-seconds", "0"])
    assert r.returncode != 0
    assert "unknown option 'no_such_option'" in r.stderr
    assert not any(ln.startswith("{") for ln in r.stdout.splitlines())
