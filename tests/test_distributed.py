"""CPU: the multi-process harness of bench.py (one rank per GPU, replicas; gloo carries the
barrier and the max/sum over ranks) with world_size 2."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

from conftest import ROOT

pytestmark = pytest.mark.cpu


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_dist_world2(tmp_path):
    script = tmp_path / "w.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, json
        sys.path.insert(0, {ROOT!r})
        from bench import Dist
        d = Dist(2)
        d.barrier()
        mx = d.max(1.5 + d.rank)
        sm = d.sum(10 * (d.rank + 1))
        # one file per rank: two ranks printing to one pipe can interleave their lines
        open(os.path.join({str(tmp_path)!r}, f"r{{d.rank}}.json"), "w").write(
            json.dumps({{"rank": d.rank, "world": d.world, "max": mx, "sum": sm}}))
    """))
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    outs = [json.loads((tmp_path / f"r{i}.json").read_text()) for i in range(2)]
    assert sorted(o["rank"] for o in outs) == [0, 1]
    for o in outs:
        assert o["world"] == 2 and o["max"] == 2.5 and o["sum"] == 30.0


def test_bench_launcher_dry_run_world2():
    """`python bench.py --gpus 2` starts its own two ranks (no torch.distributed.run) and
    rank 0 prints one line with n_gpus 2 and the summed value (host placeholder step)."""
    import json
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4",
                        "--warmup", "1", "--dry-run", "--streams", "8"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    o = lines[0]
    assert o["n_gpus"] == 2 and o["dry_run"] and o["config"]["global_batch"] == 16
    assert o["value"] == pytest.approx(2 * 4 * 8 / (o["ms_per_step"] * 4 / 1000.0), rel=0.02)


def test_bench_launcher_fails_fast_when_a_rank_dies():
    """A rank that exits with an error takes the job down at once: the launcher polls its
    children and stops the sibling waiting in the barrier (instead of leaving it there until
    the process-group timeout), and returns the failing rank's status."""
    import time
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3", "--steps", "2",
                        "--warmup", "1", "--dry-run", "--dry-run-fail-rank", "1"],
                       capture_output=True, text=True, timeout=200, env=env)
    assert r.returncode != 0
    assert "rank 1 exited" in r.stderr, r.stderr[-2000:]
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert time.time() - t0 < 120


def test_bench_rejects_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run"],
                       capture_output=True, text=True, timeout=120, env=env)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_launcher_dry_run_stagger_world2():
    """The served config-4 line under the launcher (`--gpus 2 --stagger --streams 8
    --dry-run`): both ranks come up, the line carries the served shape (8 scheduled streams
    per rank, 16 in all)."""
    import json
    env = dict(os.environ, OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2",
                        "--warmup", "1", "--dry-run", "--stagger", "--streams", "8"],
                       capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(l) for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    o = lines[0]
    assert o["n_gpus"] == 2 and o["config"]["served"] and o["config"]["global_batch"] == 16
    assert o["rank_cpus"] >= 2


def test_gpu_local_cpus_from_sysfs(tmp_path, monkeypatch):
    """Rank affinity (bench.pin_rank): HIP device i = the i-th GPU node of the KFD topology
    (after *_VISIBLE_DEVICES), its PCI function's local_cpulist gives the CPUs; a missing
    tree gives None (no pinning)."""
    sys.path.insert(0, ROOT)
    import bench
    nodes = tmp_path / "class/kfd/kfd/topology/nodes"
    # node 0: a CPU node; nodes 1, 2: GPUs at 0000:05:00.0 and 0001:85:00.0
    for i, props in enumerate(["simd_count 0\n", "simd_count 1024\nlocation_id 1280\ndomain 0\n",
                               "simd_count 1024\nlocation_id 34048\ndomain 1\n"]):
        (nodes / str(i)).mkdir(parents=True)
        (nodes / str(i) / "properties").write_text(props)
    for bdf, cl in (("0000:05:00.0", "0-3,8-9\n"), ("0001:85:00.0", "16-19\n")):
        (tmp_path / "bus/pci/devices" / bdf).mkdir(parents=True)
        (tmp_path / "bus/pci/devices" / bdf / "local_cpulist").write_text(cl)
    for v in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        monkeypatch.delenv(v, raising=False)
    assert bench.gpu_local_cpus(0, str(tmp_path)) == {0, 1, 2, 3, 8, 9}
    assert bench.gpu_local_cpus(1, str(tmp_path)) == {16, 17, 18, 19}
    monkeypatch.setenv("HIP_VISIBLE_DEVICES", "1")
    assert bench.gpu_local_cpus(0, str(tmp_path)) == {16, 17, 18, 19}
    assert bench.gpu_local_cpus(0, str(tmp_path / "nope")) is None


def test_host_weights_shared_mapping_world2(tmp_path):
    """bench.host_weights with 2 ranks: local rank 0 generates the seeded weights into
    /dev/shm, rank 1 maps them read-only; both see the bytes synth_weights makes alone, and
    the file is gone afterwards."""
    script = tmp_path / "hw.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys, json, hashlib
        sys.path.insert(0, {ROOT!r})
        sys.path.insert(0, os.path.join({ROOT!r}, "voxtral.c_amd"))
        from bench import Dist, host_weights
        from vox_weights import TINY, synth_weights
        d = Dist(2)
        w, how = host_weights(TINY, 3, d)
        ref = synth_weights(TINY, seed=3)
        same = all((w.bf16(k) == ref.bf16(k)).all() for k in ref.t)
        d.barrier()
        left = [f for f in os.listdir("/dev/shm") if f.startswith("vox_bench_w_" + os.environ["MASTER_PORT"])]
        open(os.path.join({str(tmp_path)!r}, f"r{{d.rank}}.json"), "w").write(
            json.dumps({{"same": bool(same), "how": how, "left": left}}))
    """))
    port = free_port()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(port), str(script)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    import json
    for i in range(2):
        o = json.loads((tmp_path / f"r{i}.json").read_text())
        assert o["same"] and not o["left"], o
        assert o["how"] in ("one shared read-only mapping per node", "per rank"), o
