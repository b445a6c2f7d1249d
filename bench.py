#!/usr/bin/env python3
"""Benchmark: decoder tokens/s + encoder RTF, Voxtral-Mini-4B-Realtime bf16 on MI355X.

Workload (BASELINE.json configs[1], "single stream, batch encoder + greedy decode"):
one `vox_transcribe_audio` pass over an 11.0 s clip shaped exactly like the reference's
samples/jfk.wav run -- encoder chunks of 1355, 140 and 1 mel frames (one-shot feed,
flush padding, vox_mel_finish; voxtral.c:1388-1401, 1640-1667), a 38-row decoder
prefill and 148 further greedy steps (149 tokens, as the reference CPU run in
BASELINE.md section 2).  A bench "step" is one such transcription.  Weights are seeded
random values of the exact architecture (no checkpoint offline) and the log-mel input is
synthetic; both are resident in HBM before timing.  Greedy decoding runs the full 149
steps regardless of EOS so the work per step is fixed.

Metric: value = decoder tokens/s summed over ranks (prefill excluded, as voxtral.c:
1363-1368 reports it) = total greedy steps / max over ranks of decode time.
encoder_rtf = encoder time / audio time (conv stem + encoder + adapter, voxtral.c:842-940).

Multi-GPU: one process per GPU, each an independent replica with its own stream(s)
(streams shard embarrassingly, SURVEY.md 8e: no collective on the data path); gloo carries
only the barrier and the max/sum over ranks.  Under torch.distributed.run the ranks come
from the environment (WORLD_SIZE must equal --gpus); `python bench.py --gpus N` without it
starts the N rank processes itself (before anything touches a GPU) and relays rank 0's line.
`--dry-run` runs the same harness with a host-only placeholder step (no GPU, no model): it
exists so the CPU tests can exercise the launcher and the over-ranks reduction.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd"))

import numpy as np  # noqa: E402

JFK_CHUNKS = [1355, 140, 1]      # mel frames per encoder call
AUDIO_SECONDS = 176000 / 16000.0  # samples/jfk.wav
HBM_PEAK_GBS = 8000.0            # MI355X_MICROARCH.md chip table (spec)
MFMA_BF16_TFLOPS = 2500.0        # dense bf16 MFMA peak (no sparsity), MI355X_MICROARCH.md
MPS_TOK_S = 1000.0 / 23.5        # M3 Max MPS decoder step, short clip (README.md:323)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3, help="timed transcriptions")
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=8, help="oracle decode steps in the CPU sample")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--streams", type=int, default=1,
                    help="config 4: streams per GPU decoded together (batched weight reads)")
    ap.add_argument("--q8", action="store_true",
                    help="config 5: Q8 weights (the quantize.py layout, quantised from the seeded bf16 set)")
    ap.add_argument("--streaming", action="store_true",
                    help="config 3: raw audio fed in -I-sized pieces through the device mel + chunked encoder")
    ap.add_argument("--audio-seconds", type=float, default=180.0, help="config 3 audio length")
    ap.add_argument("--interval", type=float, default=0.5, help="config 3 -I interval (s)")
    ap.add_argument("--clip-seconds", type=float, default=0.0,
                    help="config 2's long clips (e.g. 59.75): one vox_transcribe_audio pass over synthetic audio "
                         "of this length (one-shot feed through the device mel, flush, finish)")
    ap.add_argument("--stagger", action="store_true",
                    help="config 4 as a server: --streams S streams on the C host's per-GPU scheduler "
                         "(vh_sched_*), fed -I 0.5 pieces of the 7 sample lengths cycled, staggered starts")
    ap.add_argument("--serve-seconds", type=float, default=120.0,
                    help="--stagger: audio each stream serves (clips back to back)")
    ap.add_argument("--serve-end", choices=["common", "per-stream"], default="common",
                    help="--stagger: 'common' -- clips start until one common end tick (2 x serve-seconds + "
                         "streams - 1 ticks, so a stream serves serve-seconds on average), where every live "
                         "clip is finished and drained: all streams live from the last start to the end; "
                         "'per-stream' -- each stream until it has served serve-seconds (whole clips: the "
                         "streams end apart, a long tail at low occupancy)")
    ap.add_argument("--serve-fresh-streams", action="store_true",
                    help="--stagger: vh_stream_init / free for every clip instead of reusing a slot's stream "
                         "through vh_stream_reset")
    ap.add_argument("--serve-step-cap", type=int, default=8,
                    help="--stagger: greedy steps per stream and scheduler run (vh_sched_set_step_cap; 0 = "
                         "drain every run): a stream's bursts (prompt, flush padding) ride in full batched "
                         "steps over the next runs")
    ap.add_argument("--kv-fp16", action="store_true",
                    help="the reference's fp16 decoder KV cache (VOX_DECODER_KV_FP16): IEEE half K/V rings")
    ap.add_argument("--long-context", type=int, default=0,
                    help="long-context decode line: prime the decoder KV to this many positions (8192 = the "
                         "full window), then time --long-steps greedy steps")
    ap.add_argument("--long-steps", type=int, default=200, help="--long-context: timed steps (>= 100)")
    ap.add_argument("--dry-run", action="store_true",
                    help="harness check without a GPU: placeholder host step, same launcher and JSON")
    ap.add_argument("--dry-run-fail-rank", type=int, default=-1,
                    help="(tests) with --dry-run, this rank exits with an error before the first barrier")
    return ap.parse_args()


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n):
    """One process per GPU, started here before any GPU call in this process (a parent
    that touched the GPU must not fork/exec workers).  Each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / MASTER_* like torch.distributed.run would set; rank 0 prints the line."""
    port = free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    # poll every rank: the first one that fails takes its siblings down (they would
    # otherwise wait in a barrier for the dead rank until the process-group timeout)
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            r = p.poll()
            if r is None:
                continue
            live.remove(p)
            if r != 0 and rc == 0:
                rc = r
                print(f"bench.py: rank {procs.index(p)} exited with {r}; stopping the other ranks",
                      file=sys.stderr, flush=True)
                for q in live:
                    q.terminate()
                deadline = time.time() + 10
                for q in live:
                    try:
                        q.wait(timeout=max(0.1, deadline - time.time()))
                    except subprocess.TimeoutExpired:
                        q.kill()
                        q.wait()
                live = []
                break
        if live:
            time.sleep(0.05)
    return rc


GLOO_TIMEOUT_S = 600   # a rank lost mid-run ends the job within this bound, not torch's default


class Dist:
    def __init__(self, n):
        self.rank = int(os.environ.get("RANK", "0"))
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        if self.world != n:
            raise SystemExit(f"bench.py: WORLD_SIZE={self.world} but --gpus {n}")
        self.torch = None
        self.host = {}
        if self.world > 1:
            import datetime

            import torch
            import torch.distributed as dist
            self.torch, self.dist = torch, dist
            dist.init_process_group("gloo", timeout=datetime.timedelta(seconds=GLOO_TIMEOUT_S))

    def barrier(self):
        if self.torch is not None:
            self.dist.barrier()

    def max(self, x):
        if self.torch is None:
            return x
        t = self.torch.tensor([float(x)], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def min(self, x):
        if self.torch is None:
            return x
        t = self.torch.tensor([float(x)], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MIN)
        return float(t.item())

    def sum(self, x):
        if self.torch is None:
            return x
        t = self.torch.tensor([float(x)], dtype=self.torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t.item())


def emit(d, out):
    """rank 0 prints the line; multi-rank runs also say how each rank's host side was set up"""
    if d.world > 1 and d.host:
        out["rank_host"] = d.host
    if d.rank == 0:
        print(json.dumps(out), flush=True)


def parse_cpulist(text):
    """'0-3,8,10-11' -> {0, 1, 2, 3, 8, 10, 11}"""
    cpus = set()
    for part in text.strip().split(","):
        if not part:
            continue
        a, _, b = part.partition("-")
        cpus.update(range(int(a), int(b or a) + 1))
    return cpus


def gpu_local_cpus(index, sysfs="/sys"):
    """The host CPUs nearest HIP device `index` (before any GPU call): HIP numbers the GPU
    nodes of the KFD topology in node order (after ROCR / HIP_VISIBLE_DEVICES), and a node's
    PCI function lists its local CPUs.  None when any of that is unknown."""
    try:
        base = os.path.join(sysfs, "class/kfd/kfd/topology/nodes")
        gpus = []
        for node in sorted(os.listdir(base), key=int):
            props = {}
            for line in open(os.path.join(base, node, "properties")):
                k, _, v = line.partition(" ")
                props[k] = v.strip()
            if int(props.get("simd_count", "0")) > 0:
                gpus.append(props)
        for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
            vis = os.environ.get(var, "").strip()
            if vis:
                gpus = [gpus[int(x)] for x in vis.split(",")]
        p = gpus[index]
        loc, dom = int(p["location_id"]), int(p.get("domain", "0"))
        bdf = f"{dom:04x}:{loc >> 8:02x}:{(loc >> 3) & 31:02x}.{loc & 7}"
        return parse_cpulist(open(os.path.join(sysfs, "bus/pci/devices", bdf, "local_cpulist")).read())
    except (OSError, ValueError, KeyError, IndexError):
        return None


def pin_rank(d):
    """One rank per GPU: keep the rank's host threads (scheduler, device mel feeds, launches)
    on the CPUs nearest its GPU (VOX_BENCH_AFFINITY=0: off).  Returns what was done."""
    if d.world == 1 or os.environ.get("VOX_BENCH_AFFINITY") == "0" or os.environ.get("VOX_BENCH_SHARE_GPU") == "1":
        return None
    near = gpu_local_cpus(d.local)
    if not near:
        return None
    cpus = near & os.sched_getaffinity(0)
    if len(cpus) < 2:
        return None
    os.sched_setaffinity(0, cpus)
    return f"{len(cpus)} CPUs local to GPU {d.local}"


def host_weights(cfg, seed, d):
    """The seeded synthetic weights, one host copy per node: local rank 0 generates them into
    a file in /dev/shm, the other ranks map it read-only, and the file is unlinked as soon as
    every rank has mapped it (the mappings keep the pages until each rank has uploaded).  A
    single rank, or a /dev/shm too small, generates privately.  Returns (weights, how)."""
    from vox_weights import synth_elems, synth_weights, weights_over_buffer
    total = synth_elems(cfg)
    shm = "/dev/shm"
    ok = d.world > 1
    if ok:
        try:
            st = os.statvfs(shm)
            ok = st.f_bavail * st.f_frsize > total * 2 + (1 << 30)
        except OSError:
            ok = False
    ok = d.min(1.0 if ok else 0.0) > 0.5   # every rank agrees (all use the same node's /dev/shm)
    if not ok:
        return synth_weights(cfg, seed=seed), "per rank"
    path = os.path.join(shm, f"vox_bench_w_{os.environ.get('MASTER_PORT', '0')}_{seed}.bin")
    if d.local == 0:
        mm = np.memmap(path + ".tmp", dtype=np.uint16, mode="w+", shape=(total,))
        w = synth_weights(cfg, seed=seed, buf=mm)
        mm.flush()
        os.rename(path + ".tmp", path)
    d.barrier()
    if d.local != 0:
        w = weights_over_buffer(cfg, np.memmap(path, dtype=np.uint16, mode="r", shape=(total,)))
    d.barrier()
    if d.local == 0:
        os.unlink(path)
    return w, "one shared read-only mapping per node"


def transcribe(st, mel_dev, n_mel):
    """One vox_transcribe_audio-shaped pass; returns per-phase wall times (s)."""
    st.reset()
    t0 = time.perf_counter()
    off = 0
    for n in JFK_CHUNKS:
        st.encode_mel_device(mel_dev.ptr + off * n_mel * 4, n)
        off += n
    t1 = time.perf_counter()
    first = st.decode(max_steps=1, stop_at_eos=False)
    t2 = time.perf_counter()
    rest = st.decode(stop_at_eos=False)
    t3 = time.perf_counter()
    return {"enc": t1 - t0, "prefill": t2 - t1, "steps": len(rest), "step_s": t3 - t2,
            "tokens": np.concatenate([first, rest])}


def transcribe_batch(batch, streams, mel_dev, n_mel):
    """config 4: S jfk-shaped transcriptions per GPU, encoders one after another, each
    stream's prefill + first token alone, then every stream's greedy steps batched."""
    t0 = time.perf_counter()
    for i, st in enumerate(streams):
        st.reset()
        off = 0
        for n in JFK_CHUNKS:
            st.encode_mel_device(mel_dev[i].ptr + off * n_mel * 4, n)
            off += n
    t1 = time.perf_counter()
    first = [st.decode(max_steps=1, stop_at_eos=False) for st in streams]
    t2 = time.perf_counter()
    rest = batch.decode(streams, max_steps=1 << 16, stop_at_eos=False)
    t3 = time.perf_counter()
    return {"enc": t1 - t0, "prefill": t2 - t1, "steps": sum(len(r) for r in rest), "step_s": t3 - t2,
            "tokens": [np.concatenate([f, r]) for f, r in zip(first, rest)]}


def cpu_baseline(cfg, weights, mel, n_steps, q8=False):
    """The CPU restatement (oracle/, the reference's algorithm) timed on this host on a
    bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import vox_oracle
    threads = host_threads()
    om = vox_oracle.OracleModel(cfg, weights)
    st = vox_oracle.OracleStream(om)
    vox_oracle.set_threads(threads)        # sgemm threads for the M>1 encoder/prefill
    t0 = time.perf_counter()
    off = 0
    for n in JFK_CHUNKS:
        st.encode_mel(mel[off:off + n])
        off += n
    t1 = time.perf_counter()
    st.decode(max_steps=1, stop_at_eos=False)   # prefill + first token
    vox_oracle.set_threads(1)              # the reference decode GEMV is single-threaded
    t2 = time.perf_counter()
    st.decode(max_steps=n_steps, stop_at_eos=False)
    t3 = time.perf_counter()
    st.close()
    om.close()
    ms_step = (t3 - t2) * 1000.0 / n_steps
    return {"value": round(1000.0 / ms_step, 3), "unit": "tokens/s", "cores": 1, "kind": "port",
            "sample": (f"oracle/ CPU restatement, full Voxtral-4B shapes: {n_steps} greedy decode "
                       f"steps after the 38-row prefill (single-threaded "
                       + ("q8 GEMV as voxtral_kernels.c:277-318" if q8 else "bf16 GEMV as voxtral_kernels.c:154-195")
                       + f"); encoder = the 3 jfk chunks with {threads}-thread OpenBLAS sgemm"),
            "ms_per_token": round(ms_step, 2),
            "encoder_rtf": round((t1 - t0) / AUDIO_SECONDS, 4),
            "encoder_threads": threads, "cpu_model": cpu_model(), "host_cpus": len(os.sched_getaffinity(0))}


def host_threads():
    """nproc (the CPUs this process may run on), capped by OMP_NUM_THREADS when the host
    sets it: the GPU box exports 16, its share of a machine whose nproc counts every CPU."""
    n = len(os.sched_getaffinity(0))
    cap = os.environ.get("OMP_NUM_THREADS", "")
    return max(1, min(n, int(cap))) if cap.isdigit() and int(cap) > 0 else n


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def gemm_planes():
    """bf16 activation planes the M > 1 GEMMs issue per useful MFMA (vox_hip_set_gemm_planes:
    3 by default = exact f32 activations, 2 = hi + lo)"""
    import vox_hip
    return vox_hip.gemm_planes()


def encoder_dtype():
    np_ = gemm_planes()
    return (f"f32 activations as {np_} bf16 planes x bf16 weights on MFMA, f32 accumulate"
            + (" (exact)" if np_ == 3 else " (~2^-18 relative per activation)"))


def encoder_flops(cfg, mel_chunks):
    """Useful FLOPs of one stream_run_encoder pass over the given mel chunks (conv stem,
    encoder layers incl. windowed attention, adapter), following the
    stride-2 residual and the 4-row downsample carry of voxtral.c:653-692, 868-934."""
    MB, ED, H, hd, EH = cfg.mel_bins, cfg.enc_dim, cfg.enc_heads, cfg.enc_head_dim, cfg.enc_hidden
    EQ, EKV, D = H * hd, cfg.enc_kv_heads * hd, cfg.dec_dim
    per_row = 2 * ED * (EQ + 2 * EKV) + 2 * EQ * ED + 2 * ED * 2 * EH + 2 * EH * ED
    res = pos = carry = 0
    fl = 0.0
    for n in mel_chunks:
        fl += 2.0 * n * (MB * 3) * ED                      # conv0 (k3 s1)
        tot = res + n
        res = tot & 1
        t1 = (tot - res) // 2
        fl += 2.0 * t1 * (ED * 3) * ED                     # conv1 (k3 s2)
        for i in range(t1):                                # layers: projections + attention
            keys = min(pos + i + 1, cfg.enc_window)
            fl += cfg.enc_layers * (per_row + 4.0 * H * hd * keys)
        pos += t1
        usable = (carry + t1) // 4
        carry = (carry + t1) % 4
        fl += 2.0 * usable * (4 * ED * D + D * D)          # adapter
    return fl


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    d = Dist(args.gpus)
    if args.dry_run:
        return dry_run(args, d)
    affinity = pin_rank(d)
    import vox_hip
    from vox_weights import VOXTRAL_4B, quantize_q8
    # VOX_BENCH_SHARE_GPU=1: every rank on device 0 -- a rehearsal of the multi-rank path
    # (launcher, barrier, max / sum over ranks) on a one-GPU box; its timings mean nothing
    vox_hip.init(device=0 if os.environ.get("VOX_BENCH_SHARE_GPU") == "1" else d.local)
    cfg = VOXTRAL_4B

    w, w_how = host_weights(cfg, args.seed, d)
    if args.q8:
        w = quantize_q8(w)
    model = vox_hip.Model(cfg, w)
    d.host = {"cpu_affinity": affinity, "host_weights": w_how}
    if args.kv_fp16:
        model.set_kv_fp16(True)  # before any stream exists
    keep_host = d.rank == 0 and d.world == 1 and not args.no_cpu_baseline
    if not keep_host:
        del w
        w = None
    st = vox_hip.Stream(model)
    rng = np.random.default_rng(1234 + d.rank)
    mel = rng.uniform(-0.6, 1.4, size=(sum(JFK_CHUNKS), cfg.mel_bins)).astype(np.float32)
    mel_dev = vox_hip.DeviceArray(mel)
    if args.long_context > 0:
        return bench_long(args, d, cfg, model, st)
    if args.stagger:
        return bench_serve(args, d, cfg, model, st)
    if args.streams > 1:
        return bench_streams(args, d, cfg, model, st, mel, mel_dev, rng)
    if args.streaming or args.clip_seconds > 0:
        return bench_streaming(args, d, cfg, model, st)

    for _ in range(args.warmup):
        transcribe(st, mel_dev, cfg.mel_bins)

    # HIP events recorded by each W1|W3 launch's own dispatch packet (hipExtLaunchKernel) on
    # the stream's queue; profiled decode steps are launched eagerly (a graph cannot carry
    # dispatch events), which runs as fast as the graph replay
    st.set_profiling(True)
    if os.environ.get("VOX_BENCH_MAPS"):
        # the process's mappings, to put a crash's frame addresses to library + offset
        # (the rocprofv3 SIGSEGV of DESIGN.md 6; tools/run/r4_d.sh)
        with open("/proc/self/maps") as f, open(os.environ["VOX_BENCH_MAPS"], "w") as o:
            o.write(f.read())
    runs = []
    d.barrier()
    st.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runs.append(transcribe(st, mel_dev, cfg.mel_bins))
    st.sync()
    t1 = time.perf_counter()
    d.barrier()
    prof = st.profile()
    st.set_profiling(False)
    # encoder_rtf is the exact figure (3 planes: f32-exact activations, the reference's sgemm
    # precision); the approximate 2-plane split is timed after the timed region as an extra key
    enc_2plane = None
    if gemm_planes() == 3:
        vox_hip.set_gemm_planes(2)
        transcribe(st, mel_dev, cfg.mel_bins)
        d.barrier()
        e2 = [transcribe(st, mel_dev, cfg.mel_bins)["enc"] for _ in range(args.steps)]
        enc_2plane = d.max(sum(e2)) / (AUDIO_SECONDS * args.steps)
        vox_hip.set_gemm_planes(3)

    wall = d.max(t1 - t0)
    steps_local = sum(r["steps"] for r in runs)
    dec_s = d.max(sum(r["step_s"] for r in runs))
    steps_all = d.sum(steps_local)
    enc_s = d.max(sum(r["enc"] for r in runs))
    prefill_s = d.max(sum(r["prefill"] for r in runs))
    tok_s = steps_all / dec_s

    # roofline of the dominant kernel: the fused RMSNorm*(1+ada) -> W1|W3 GEMV -> SiLU*up
    # (26 launches per token, 43% of the decode bytes; DESIGN.md "Roofline")
    D, H = cfg.dec_dim, cfg.dec_hidden
    wb = 1 if args.q8 else 2
    # W1|W3 (+ Q8 row scales) + x, norm w, ada in + gate out
    w13_bytes = 2 * H * D * wb + (2 * H * 4 if args.q8 else 0) + D * 4 * 3 + H * 4
    avg_ms = prof["avg_ms"] if prof["launches"] else float("nan")
    achieved = w13_bytes / (avg_ms * 1e-3) / 1e9 if prof["launches"] else None
    traffic = None
    # W1|W3 HBM bytes per launch from the PMC passes (tools/pmc.sh, tools/pmc_q8.sh)
    pmc = os.path.join(ROOT, "profiles", "pmc_w13_q8_traffic.json" if args.q8 else "pmc_w13_traffic.json")
    if os.path.exists(pmc):
        traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")

    out = {
        "metric": ("decoder tokens/sec + encoder RTF, Voxtral-4B q8 (config 5) at 1/2/4/8 MI355X" if args.q8
                   else "decoder tokens/sec + encoder RTF, Voxtral-4B bf16 at 1/2/4/8 MI355X"),
        "value": round(tok_s, 2),
        "unit": "tokens/s",
        "n_gpus": d.world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall * 1000.0 / args.steps, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(tok_s / d.world / MPS_TOK_S, 2),
        "vs_baseline_ref": "per-GPU tok/s vs 42.6 tok/s, Apple M3 Max MPS, README.md:323 (BASELINE.md 1)",
        "dtype": "f32",
        "weights_dtype": "q8 (int8 + f32 row scales, quantize.py)" if args.q8 else "bf16",
        "data": "synthetic (seeded random weights of the exact architecture; synthetic log-mel)",
        "config": {"workload": "jfk.wav one-shot transcription shape: 1355/140/1-frame encoder "
                               "chunks, 38-row prefill, 148 greedy steps",
                   "model": "Voxtral-Mini-4B-Realtime", "global_batch": d.world, "seq_len": 149,
                   "streams_per_gpu": 1, "parallelism": f"replicas x{d.world} (no collective)"},
        "encoder_rtf": round(enc_s / (AUDIO_SECONDS * args.steps), 5),
        "encoder_dtype": encoder_dtype(),
        "encoder_rtf_2plane": round(enc_2plane, 5) if enc_2plane is not None else None,
        # k_gemmf stream-K tiles whose owner recomputed a part (the hand-off wait timed out)
        "encoder_gemm_recomputes": prof.get("gemmf_recomputes"),
        "prefill_ms": round(prefill_s * 1000.0 / args.steps, 3),
        "decoder_ms_per_token": round(dec_s * 1000.0 / max(1, steps_local), 4),
        "roofline": {"bound": "hbm", "kernel": "k_gemv<PRO_NORM_ADA,EPI_SWIGLU> (W1|W3)",
                     "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4) if achieved else None,
                     "traffic": traffic, "bytes_per_launch": w13_bytes,
                     "avg_launch_us": round(avg_ms * 1000.0, 3) if prof["launches"] else None,
                     "launches_timed": prof["launches"]},
    }
    # per-token roofline of the whole decode step: weights + the KV rows attention reads
    # (f32 K and V, positions 39..186 of the jfk schedule), SURVEY.md 8d
    L_avg = (39 + 38 + steps_local // args.steps) / 2.0
    w_tok = (6857687040 // 2) if args.q8 else 6857687040
    tok_bytes = w_tok + kv_bytes_per_position(cfg, args.kv_fp16) * L_avg
    ms_tok = dec_s * 1000.0 / max(1, steps_local)
    out["decoder_roofline"] = {"bound": "hbm", "bytes_per_token": int(tok_bytes),
                               "achieved": round(tok_bytes / (ms_tok * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                               "unit": "GB/s", "frac": round(tok_bytes / (ms_tok * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    # encoder (one-shot 1355/140/1 chunks, M = 677 rows: above the MFMA ridge): useful FLOPs
    # over the whole conv + encoder + adapter time vs the dense bf16 MFMA peak.  The GEMMs
    # issue 3 bf16 MFMAs per product (hi/mid/lo split of the f32 activations), so the
    # issued-MFMA fraction is ~3x the useful one.
    efl = encoder_flops(cfg, JFK_CHUNKS)
    enc_tf = efl / (enc_s / args.steps) / 1e12
    out["encoder_roofline"] = {"bound": "mfma", "flops_per_pass": int(efl), "achieved": round(enc_tf, 1),
                               "peak": MFMA_BF16_TFLOPS, "unit": "TFLOP/s",
                               "frac": round(enc_tf / MFMA_BF16_TFLOPS, 4), "mfma_planes": gemm_planes(),
                               "issued_frac": round(gemm_planes() * enc_tf / MFMA_BF16_TFLOPS, 4)}
    if keep_host:
        out["cpu_baseline"] = cpu_baseline(cfg, w, mel, args.cpu_steps, q8=args.q8)
    emit(d, out)
    mel_dev.free()
    st.close()
    model.close()


def kv_bytes_per_position(cfg, kv16):
    """decoder K + V bytes one attention step reads per key position (all layers): 212,992
    for f32 rings, 106,496 for IEEE half"""
    return 2 * cfg.dec_layers * cfg.dec_kv_heads * cfg.dec_head_dim * (2 if kv16 else 4)


def bench_long(args, d, cfg, model, st):
    """Long-context decode (north_star's 8192-slot rolling KV): one stream encodes enough
    synthetic mel for --long-context + --long-steps adapter rows, decodes untimed until the
    attention spans min(position + 1, window) = --long-context keys, then times --long-steps
    greedy steps (graph replay, device-held positions, the attention's key-split buckets up
    to the window's 32).  Per-token bytes = weights + K/V bytes per key x keys."""
    import vox_hip
    L, n_time = args.long_context, max(100, args.long_steps)
    rows = L + n_time + 64
    rng = np.random.default_rng(4321 + d.rank)
    mel = rng.uniform(-0.6, 1.4, size=(8 * rows, cfg.mel_bins)).astype(np.float32)
    mel_dev = vox_hip.DeviceArray(mel)
    st.reset()
    for off in range(0, mel.shape[0], 4096):
        n = min(4096, mel.shape[0] - off)
        st.encode_mel_device(mel_dev.ptr + off * cfg.mel_bins * 4, n)
    first = st.decode(max_steps=1, stop_at_eos=False)          # 38-row prefill + first token
    prompt = st.state()["kv_pos"]
    prime = max(0, L - prompt)
    st.decode(max_steps=prime, stop_at_eos=False)
    st.sync()
    pos0 = st.state()["kv_pos"]
    d.barrier()
    st.sync()
    t0 = time.perf_counter()
    ids = st.decode(max_steps=n_time, stop_at_eos=False)
    st.sync()
    t1 = time.perf_counter()
    d.barrier()
    assert len(ids) == n_time, (len(ids), n_time)
    wall = d.max(t1 - t0)
    tok_s = d.sum(len(ids)) / wall
    keys = min(L, cfg.dec_window)
    w_tok = (6857687040 // 2) if args.q8 else 6857687040
    kvb = kv_bytes_per_position(cfg, args.kv_fp16)
    tok_bytes = w_tok + kvb * keys
    ms_tok = wall * 1000.0 / len(ids)
    out = {
        "metric": "decoder tokens/sec at a full 8192-key window, Voxtral-4B bf16 (long-context decode)",
        "value": round(tok_s, 2), "unit": "tokens/s", "n_gpus": d.world, "steps": len(ids), "warmup": prime,
        "ms_per_step": round(ms_tok, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "f32", "weights_dtype": "q8" if args.q8 else "bf16",
        "kv_dtype": "f16 (IEEE half, VOX_DECODER_KV_FP16)" if args.kv_fp16 else "f32",
        "data": "synthetic (seeded random weights of the exact architecture; synthetic log-mel)",
        "config": {"workload": f"one stream primed to {L} decoder positions ({prime} untimed greedy steps after the "
                               f"prompt), then {n_time} timed greedy steps attending {keys} keys each",
                   "model": "Voxtral-Mini-4B-Realtime", "global_batch": d.world, "seq_len": keys,
                   "streams_per_gpu": 1, "parallelism": f"replicas x{d.world} (no collective)"},
        "first_timed_position": pos0, "first_token": int(first[0]) if len(first) else None,
        "decoder_roofline": {"bound": "hbm", "bytes_per_token": int(tok_bytes), "kv_bytes_per_key": kvb,
                             "achieved": round(tok_bytes / (ms_tok * 1e-3) / 1e9, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(tok_bytes / (ms_tok * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
    }
    emit(d, out)
    mel_dev.free()
    st.close()
    model.close()


def dry_run(args, d):
    """The launcher / reduction path without a GPU: every rank times `steps` placeholder
    host steps (a small numpy matmul standing in for a transcription) between the same
    barriers and reports the same aggregate fields.  Not a measurement of the engine."""
    if d.rank == args.dry_run_fail_rank:
        sys.exit(f"bench.py: rank {d.rank} failing on purpose (--dry-run-fail-rank)")
    a = np.random.default_rng(d.rank).standard_normal((256, 256)).astype(np.float32)
    for _ in range(args.warmup):
        a @ a
    d.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        a = (a @ a) / np.float32(16.0)
    t1 = time.perf_counter()
    d.barrier()
    wall = d.max(t1 - t0)
    steps_all = d.sum(args.steps * args.streams)
    out = {"metric": "bench.py harness dry run (no GPU; placeholder host step)", "value": round(steps_all / wall, 2),
           "unit": "steps/s", "n_gpus": d.world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(wall * 1000.0 / args.steps, 3), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "f32", "data": "synthetic", "dry_run": True,
           "config": {"workload": "placeholder", "global_batch": d.world * args.streams,
                      "streams_per_gpu": args.streams, "parallelism": f"replicas x{d.world} (no collective)"}}
    if args.stagger:
        # the served config-4 line's shape (bench_serve): S scheduled streams per rank
        out["config"].update({"workload": "placeholder for the served line (--stagger)", "served": True,
                              "serve_seconds": args.serve_seconds,
                              "parallelism": f"replicas x{d.world}, {args.streams} scheduled streams each"})
        out["rank_cpus"] = d.sum(len(os.sched_getaffinity(0)))
        d.host = {"cpu_affinity": pin_rank(d)}
    emit(d, out)


def synth_audio(seconds, seed):
    """Speech-band synthetic audio: noise bursts under a slow envelope plus drifting tones
    (no recording is available offline; the path's work depends only on the length)."""
    rng = np.random.default_rng(seed)
    n = int(seconds * 16000)
    t = np.arange(n) / 16000.0
    env = 0.5 + 0.5 * np.sin(2 * np.pi * 0.7 * t) * np.sin(2 * np.pi * 0.13 * t)
    x = 0.05 * rng.standard_normal(n) * env + 0.1 * env * np.sin(2 * np.pi * (180 + 60 * np.sin(0.5 * t)) * t)
    return x.astype(np.float32)


def bench_streaming(args, d, cfg, model, st):
    """config 3 (BASELINE.json configs[2]): main.c's file mode with -I <interval>
    (main.c:110-118, 200-204): the audio goes in interval-sized pieces through
    vox_stream_feed (device log-mel, incremental conv stem, chunked encoder with the
    rolling 750-row KV, adapter) with the decoder drained after every piece, then
    vox_stream_finish.  Decoding ignores EOS so the work is fixed."""
    import vox_hip
    oneshot = args.clip_seconds > 0
    if oneshot:
        # vox_transcribe_audio (voxtral.c:1388-1401): every sample in one vox_stream_feed
        args.audio_seconds = args.clip_seconds
        args.interval = args.clip_seconds
    audio = synth_audio(args.audio_seconds, 99 + d.rank)
    piece = len(audio) if oneshot else max(160, min(int(args.interval * 16000), 16000 * 60))
    secs = len(audio) / 16000.0

    class Timed:
        """the stream with its encoder / decoder calls timed (synchronised)"""
        def __init__(self, s):
            self.s, self.model, self.cfg = s, s.model, s.cfg
            self.t_enc = self.t_dec = 0.0
            self.steps = 0

        def encode_mel_device(self, ptr, n):
            t0 = time.perf_counter()
            r = self.s.encode_mel_device(ptr, n)
            self.s.sync()
            self.t_enc += time.perf_counter() - t0
            return r

        def decode(self, **kw):
            t0 = time.perf_counter()
            r = self.s.decode(**kw)
            self.t_dec += time.perf_counter() - t0
            self.steps += len(r)
            return r

    def run():
        st.reset()
        ts = Timed(st)
        sess = vox_hip.AudioSession(st, interval_s=args.interval)
        sess.s = ts
        t_mel = 0.0
        t0 = time.perf_counter()
        for i in range(0, len(audio), piece):
            a = time.perf_counter()
            sess.mel.feed(audio[i:i + piece])
            st.sync()
            t_mel += time.perf_counter() - a
            sess.real_samples += min(piece, len(audio) - i)
            sess.feed(sess.mel, stop_at_eos=False)
        sess.finish_samples(stop_at_eos=False)
        st.sync()
        wall = time.perf_counter() - t0
        sess.close()
        return {"wall": wall, "enc": ts.t_enc + t_mel, "dec": ts.t_dec, "steps": ts.steps,
                "chunks": len(sess.chunks), "chunk_frames": list(sess.chunks), "tokens": len(sess.tokens)}

    for _ in range(args.warmup):
        run()
    d.barrier()
    runs = [run() for _ in range(args.steps)]
    d.barrier()
    dec_s = d.max(sum(r["dec"] for r in runs))
    steps_all = d.sum(sum(r["steps"] for r in runs))
    enc_s = d.max(sum(r["enc"] for r in runs))
    wall = d.max(sum(r["wall"] for r in runs))
    tok_s = steps_all / dec_s
    # encoder chunk roofline: a 0.5 s chunk is ~25 encoder rows, far below the MFMA ridge
    # (SURVEY.md 8d): every chunk streams the encoder + adapter weights once (bf16 / int8)
    wb = 1 if args.q8 else 2
    eq, ekv = cfg.enc_heads * cfg.enc_head_dim, cfg.enc_kv_heads * cfg.enc_head_dim
    enc_w = cfg.enc_layers * (eq + 2 * ekv + eq + 2 * cfg.enc_hidden + cfg.enc_hidden) * cfg.enc_dim * wb
    enc_w += (4 * cfg.enc_dim + cfg.dec_dim) * cfg.dec_dim * wb
    ms_chunk = enc_s * 1000.0 / max(1, sum(r["chunks"] for r in runs))
    if oneshot:
        mode = f"{args.clip_seconds} s clip one-shot (config 2 long clip)"
        workload = (f"{args.clip_seconds} s of 16 kHz audio in one vox_stream_feed + flush + finish "
                    f"(vox_transcribe_audio): device log-mel, encoder chunks {runs[0]['chunk_frames']} mel frames "
                    f"(<= 1024-row passes), {runs[0]['steps']} greedy steps")
    else:
        mode = f"streaming -I {args.interval} (config 3)"
        workload = (f"{args.audio_seconds:.0f} s of 16 kHz audio fed in {piece}-sample pieces "
                    f"(main.c file mode, -I {args.interval}): device log-mel, {runs[0]['chunks']} encoder "
                    f"chunks, {runs[0]['steps']} greedy steps (KV to ~{runs[0]['steps'] + 40} positions)")
    out = {
        "metric": "decoder tokens/sec + encoder RTF, Voxtral-4B " + ("q8" if args.q8 else "bf16")
                  + f", {mode}, at 1/2/4/8 MI355X",
        "value": round(tok_s, 2), "unit": "tokens/s", "n_gpus": d.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall * 1000.0 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": round(tok_s / d.world / MPS_TOK_S, 2),
        "dtype": "f32", "weights_dtype": "q8" if args.q8 else "bf16",
        "data": "synthetic (seeded random weights of the exact architecture; synthetic speech-band audio)",
        "config": {"workload": workload,
                   "model": "Voxtral-Mini-4B-Realtime", "global_batch": d.world, "seq_len": runs[0]["steps"],
                   "streams_per_gpu": 1, "parallelism": f"replicas x{d.world} (no collective)"},
        "encoder_rtf": round(enc_s / (secs * args.steps), 5),
        "encoder_dtype": encoder_dtype(),
        "overall_rtf": round(wall / (secs * args.steps), 5),
        "encoder_ms_per_chunk": round(ms_chunk, 3),
        "encoder_weight_bytes_per_chunk": enc_w,
        "encoder_chunk_weight_gbs": round(enc_w / (ms_chunk * 1e-3) / 1e9, 1),
        "decoder_ms_per_token": round(dec_s * 1000.0 / max(1, steps_all / d.world), 4),
    }
    if oneshot:
        # long one-shot chunks are MFMA work: useful FLOPs of the schedule (mel + conv + encoder
        # + adapter time) against the dense bf16 peak (3 bf16 MFMAs per product: issued ~3x)
        efl = encoder_flops(cfg, runs[0]["chunk_frames"])
        tf = efl / (enc_s / args.steps) / 1e12
        out["encoder_roofline"] = {"bound": "mfma", "flops_per_pass": int(efl), "achieved": round(tf, 1),
                                   "peak": MFMA_BF16_TFLOPS, "unit": "TFLOP/s", "frac": round(tf / MFMA_BF16_TFLOPS, 4),
                                   "mfma_planes": gemm_planes(),
                                   "issued_frac": round(gemm_planes() * tf / MFMA_BF16_TFLOPS, 4)}
    else:
        # ~25-row chunks are far below the MFMA ridge: every chunk streams the encoder +
        # adapter weights once, so the bound is that byte stream at the HBM peak
        gbs = enc_w / (ms_chunk * 1e-3) / 1e9
        out["encoder_roofline"] = {"bound": "hbm", "bytes_per_chunk": enc_w, "achieved": round(gbs, 1),
                                   "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
    emit(d, out)
    st.close()
    model.close()


# the reference's 7 WAV samples (samples/jfk.wav, test_speech.wav, benchmark/night1968/*):
# their lengths in seconds; the served audio is synthetic of these lengths
SAMPLE_SECONDS = [11.0, 3.64175, 5.0000625, 15.0000625, 45.0000625, 59.7494375, 88.8899375]


def bench_serve(args, d, cfg, model, st0):
    """config 4 as a serving loop (BASELINE.json configs[3]; SURVEY.md 8d: "the 7 WAVs
    cycled, 8 per GPU, staggered starts"): S concurrent streams on this GPU, owned by the C
    host's scheduler (vh_sched_*, include/vox_hip_host.h).  Stream i starts 1 s (two ticks)
    after stream i-1 and transcribes the 7 sample lengths in turn from clip i on, a fresh
    vh_stream per clip, until a common end tick (--serve-end common: 2 x --serve-seconds + S - 1
    ticks, where every unfinished clip is finished -- its audio so far -- and drained) or until it
    has served --serve-seconds of whole clips (--serve-end per-stream).  One tick = every live
    stream feeds its next 0.5 s piece (vox_stream_feed: device mel + encoder chunk; -I 0.5),
    or flush + finish after its clip's last piece, then one vh_sched_run (prefills + batched
    greedy steps for every stream with adapter rows).  Ticks run back to back (as fast as the
    GPU goes).  Reported: aggregate ids/s over the whole loop, the tick latency (a piece's
    wait for its ids) p50 / p99, and audio served per wall second."""
    import vox_hip
    st0.close()
    S, piece = args.streams, 8000
    ctx = vox_hip.HostCtx(model)
    q = vox_hip.Scheduler(ctx, S)
    q.set_step_cap(args.serve_step_cap)
    rng = np.random.default_rng(5 + d.rank)
    clips = [synth_audio(sec, 500 + k) for k, sec in enumerate(SAMPLE_SECONDS)]

    common = args.serve_end == "common"
    pool = [[] for _ in range(S)]   # reusable vh_streams per stream slot

    def run(serve_s):
        end_tick = int(round(2 * serve_s)) + S - 1  # common end (ticks of 0.5 s)
        served = [0.0] * S
        cur = [None] * S        # [HostStream, clip index, next sample, finished]
        nxt = list(range(S))
        ids, lat, clips_done, tick = 0, [], 0, 0
        full = [0, 0.0]         # ids and wall time of the ticks in which all S streams were live
        host = [0.0, 0.0, 0.0]  # wall in the feeds, in vh_sched_run, in reading ids / retiring clips
        t_all = time.perf_counter()
        while True:
            live = False
            n_live = 0
            t0 = time.perf_counter()
            for k in range(S):
                if tick < 2 * k:             # staggered start
                    live = True
                    continue
                if cur[k] is None:
                    if (tick >= end_tick) if common else (served[k] >= serve_s):
                        continue
                    # a fresh vh_stream per clip, reused from the slot's pool (vh_stream_reset:
                    # the state vh_stream_init leaves, without its device allocations) unless
                    # --serve-fresh-streams
                    hs = pool[k].pop() if pool[k] else vox_hip.HostStream(ctx, interval_s=0.5)
                    q.attach(hs)
                    cur[k] = [hs, nxt[k] % len(clips), 0, False]
                    nxt[k] += 1
                live = True
                n_live += 1
                hs, c, pos, fin = cur[k]
                if fin:                       # finished, rows still being decoded (step cap)
                    continue
                if common and tick >= end_tick:  # the common end: the clip so far, flushed
                    hs.finish()
                    cur[k][3] = True
                elif pos < len(clips[c]):
                    hs.feed(clips[c][pos:pos + piece])
                    cur[k][2] = pos + piece
                else:
                    hs.finish()
                    cur[k][3] = True
            if not live:
                break
            t1 = time.perf_counter()
            q.run()
            t2 = time.perf_counter()
            host[0] += t1 - t0
            host[1] += t2 - t1
            tick_ids = 0
            for k in range(S):
                if cur[k] is None:
                    continue
                tick_ids += len(cur[k][0].get())
                if cur[k][3] and cur[k][0].pending() == 0:   # finished and drained: retire the clip
                    served[k] += min(cur[k][2], len(clips[cur[k][1]])) / 16000.0
                    q.detach(cur[k][0])
                    if args.serve_fresh_streams:
                        cur[k][0].close()
                    else:
                        cur[k][0].reset()
                        pool[k].append(cur[k][0])
                    cur[k] = None
                    clips_done += 1
            ids += tick_ids
            lat.append(time.perf_counter() - t0)
            host[2] += time.perf_counter() - t2
            if n_live == S:
                full[0] += tick_ids
                full[1] += lat[-1]
            tick += 1
        return {"wall": time.perf_counter() - t_all, "ids": ids, "lat": lat, "ticks": tick,
                "clips": clips_done, "audio_s": sum(served), "full_ids": full[0], "full_s": full[1],
                "host": host}

    for _ in range(args.warmup):
        run(min(args.serve_seconds, 20.0))
    q_stats0 = q.stats()
    d.barrier()
    runs = [run(args.serve_seconds) for _ in range(args.steps)]
    d.barrier()
    st = q.stats()
    for p in pool:
        for hs in p:
            hs.close()
    wall = d.max(sum(r["wall"] for r in runs))
    ids_all = d.sum(sum(r["ids"] for r in runs))
    audio_all = d.sum(sum(r["audio_s"] for r in runs))
    lat = np.array([x for r in runs for x in r["lat"]]) * 1000.0
    batch_tok = st["tokens"] - q_stats0["tokens"]
    batch_ms = st["batch_ms"] - q_stats0["batch_ms"]
    batch_steps = st["steps"] - q_stats0["steps"]
    ticks = sum(r["ticks"] for r in runs)
    out = {
        "metric": "decoder tokens/sec + encoder RTF, Voxtral-4B " + ("q8" if args.q8 else "bf16")
                  + f", {S} streams per MI355X served by the per-GPU scheduler (config 4), at 1/2/4/8 MI355X",
        "value": round(ids_all / wall, 2), "unit": "tokens/s", "n_gpus": d.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall * 1000.0 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": round(ids_all / wall / d.world / MPS_TOK_S, 2),
        "dtype": "f32", "weights_dtype": "q8" if args.q8 else "bf16",
        "data": "synthetic (seeded random weights of the exact architecture; synthetic speech-band audio "
                "of the 7 sample lengths)",
        "config": {"workload": f"{S} streams per GPU, "
                               + (f"clips starting until a common end after {args.serve_seconds:.0f} s of audio per "
                                  "stream on average (every clip then finished and drained)" if common else
                                  f"each serving {args.serve_seconds:.0f} s of audio as whole clips")
                               + f" of the 7 sample lengths {[round(x, 2) for x in SAMPLE_SECONDS]} s cycled (from "
                               "clip i), fed in 0.5 s pieces (-I 0.5), starts staggered by 1 s; one vh_sched_run "
                               "per tick"
                               + (f", at most {args.serve_step_cap} greedy steps per stream and run (a finished clip "
                                  "drains over the next ticks before the stream's next clip)"
                                  if args.serve_step_cap > 0 else ""),
                   "model": "Voxtral-Mini-4B-Realtime", "global_batch": S * d.world, "streams_per_gpu": S,
                   "parallelism": f"replicas x{d.world}, {S} scheduled streams each",
                   "serve_end": args.serve_end, "serve_step_cap": args.serve_step_cap,
                   "streams_per_clip": "fresh (vh_stream_init)" if args.serve_fresh_streams
                                       else "reused (vh_stream_reset)"},
        "value_is": "all ids generated / wall time of the serving loop (mel, encoder, prefill and decode included)",
        "tick_latency_ms": {"p50": round(float(np.percentile(lat, 50)), 3),
                            "p99": round(float(np.percentile(lat, 99)), 3), "max": round(float(lat.max()), 3)},
        "audio_seconds_per_wall_second": round(audio_all / wall, 2),
        "overall_rtf_per_stream": round(wall / (audio_all / d.world / S), 5),
        "clips": sum(r["clips"] for r in runs),
        # the ticks in which every one of the S streams was live (the stagger ramp and the tail
        # of the longest clips excluded): the scheduler's rate at full occupancy
        "all_streams_live": {"ids": sum(r["full_ids"] for r in runs),
                             "s": round(sum(r["full_s"] for r in runs), 3),
                             "ids_per_s": round(sum(r["full_ids"] for r in runs) / max(1e-9, sum(r["full_s"] for r in runs)), 1),
                             "share_of_wall": round(sum(r["full_s"] for r in runs) / max(1e-9, sum(r["wall"] for r in runs)), 3)},
        "batched_decode": {"ids": batch_tok, "ms": round(batch_ms, 1),
                           "ids_per_s": round(batch_tok / max(1e-9, batch_ms * 1e-3), 1),
                           "steps": batch_steps, "rows_per_step": round(batch_tok / max(1, batch_steps), 2),
                           "graph_captures": st["captures"] - q_stats0["captures"],
                           "graph_captures_per_tick": round((st["captures"] - q_stats0["captures"]) / max(1, ticks), 4),
                           "prefill_passes": st["prefill_passes"] - q_stats0["prefill_passes"],
                           "prefilled_streams": st["prefills"] - q_stats0["prefills"],
                           "ticks": ticks},
        # with the scheduler's overlap (VOX_HIP_SCHED_OVERLAP, default on) the passes run beside
        # the batched steps and their ms count the enqueue only
        "encoder_passes": {"ms": round(st["enc_ms"] - q_stats0["enc_ms"], 1),
                           "passes": st["enc_batches"] - q_stats0["enc_batches"],
                           "overlapped": os.environ.get("VOX_HIP_SCHED_OVERLAP", "1") != "0"},
        # time inside vh_sched_run (encoder pass, prefills, steps) vs the rest of the ticks
        # (feeding pieces: device mel, conv stems queued; reading ids)
        "scheduler_run_ms": round(st["run_ms"] - q_stats0["run_ms"], 1),
        # the tick loop's wall split: feeding the pieces (device mel, conv stems queued), the
        # scheduler run, reading ids and retiring finished clips
        "tick_wall_ms": {k: round(1000.0 * sum(r["host"][i] for r in runs), 1)
                         for i, k in enumerate(("feed", "run", "collect"))},
    }
    emit(d, out)
    q.close()
    ctx.close()
    model.close()


def bench_streams(args, d, cfg, model, st0, mel0, mel_dev0, rng):
    """config 4 (BASELINE.json configs[3]): S concurrent streams per GPU, batched decode."""
    import vox_hip
    S = args.streams
    streams = [st0] + [vox_hip.Stream(model) for _ in range(S - 1)]
    mels = [mel_dev0] + [vox_hip.DeviceArray(rng.uniform(-0.6, 1.4, size=mel0.shape).astype(np.float32))
                         for _ in range(S - 1)]
    batch = vox_hip.Batch(model, S)
    for _ in range(args.warmup):
        transcribe_batch(batch, streams, mels, cfg.mel_bins)
    runs = []
    d.barrier()
    streams[0].sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runs.append(transcribe_batch(batch, streams, mels, cfg.mel_bins))
    t1 = time.perf_counter()
    d.barrier()
    wall = d.max(t1 - t0)
    dec_s = d.max(sum(r["step_s"] for r in runs))
    steps_all = d.sum(sum(r["steps"] for r in runs))
    tok_s = steps_all / dec_s
    enc_s = d.max(sum(r["enc"] for r in runs))
    out = {
        "metric": "decoder tokens/sec + encoder RTF, Voxtral-4B " + ("q8" if args.q8 else "bf16")
                  + f", {S} streams per MI355X (config 4), at 1/2/4/8 MI355X",
        "value": round(tok_s, 2), "unit": "tokens/s", "n_gpus": d.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(wall * 1000.0 / args.steps, 3),
        "higher_is_better": True, "scaling": "weak", "vs_baseline": round(tok_s / d.world / MPS_TOK_S, 2),
        "dtype": "f32", "weights_dtype": "q8" if args.q8 else "bf16",
        "data": "synthetic (seeded random weights of the exact architecture; synthetic log-mel per stream)",
        "config": {"workload": f"{S} jfk.wav-shaped transcriptions per GPU; per-stream encoder and prefill, "
                               "greedy steps batched across the streams (one weight read per step)",
                   "model": "Voxtral-Mini-4B-Realtime", "global_batch": S * d.world, "seq_len": 149,
                   "streams_per_gpu": S, "parallelism": f"replicas x{d.world}, {S} streams each"},
        "encoder_rtf": round(enc_s / (AUDIO_SECONDS * S * args.steps), 5),
        "encoder_dtype": encoder_dtype(),
        "decoder_ms_per_batched_step": round(dec_s * 1000.0 / max(1, steps_all / d.world / S), 4),
    }
    emit(d, out)
    batch.close()
    for m_ in mels:
        m_.free()
    for s_ in streams:
        s_.close()
    model.close()


if __name__ == "__main__":
    main()
