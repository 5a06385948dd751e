"""RTFx benchmark of the MI355X Whisper backend (BASELINE.json metric).

Workload (BASELINE.json configs[2], one GPU): Whisper-large-v3 dimensions, bf16
weights/activations (f32 accumulation), batch of 8 synthetic 30 s 16 kHz chunks
(BASELINE.md §3 signal, seeds 1000+i), greedy decode with language "en",
<|notimestamps|>, a 4-token prompt and 128 forced decode steps (EOT ignored:
random-init weights never stop).  Weights are random-init from the shared seeded
PRNG (no checkpoints offline).  One "step" = one batched call through the C ABI
(spt_transcribe_batch, BASELINE.md:48's span): host PCM -> H2D -> log-mel -> encoder ->
cross K/V -> 132 decoder passes -> tokens and text on the host.  `value` is that rate;
`value_device_resident` is the same call on PCM already in HBM
(spt_transcribe_batch_device).

--gpus N (BASELINE.json configs[3]): one process per GPU.  Launched by torchrun (WORLD_SIZE
set) each rank runs here; launched plainly, this process starts the N ranks itself
(torch.distributed.run, before touching the GPU) and exits with their status.  Each rank
transcribes its own shard of 8 utterances per step (weak scaling, no data-path collective);
rank 0 loads the weights and one RCCL broadcast writes them straight into every other rank's
weight arena; the timed region is bracketed by barriers and the max over ranks is reported.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

MODEL_SPEC = "synthetic:large-v3"
CHUNK_S = 30.0
PROMPT_LEN = 4
N_STEPS = 128
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8.0 TB/s HBM3E (spec)
MFMA_PEAK_BF16_TFS = 2500.0  # dense bf16
FP32_PEAK_TFS = 157.3        # f32 MFMA = vector rate
MFMA_PEAK_F16_TFS = 2500.0   # dense fp16 (same rate as bf16)
PK_SPEC = "synthetic:parakeet-tdt-0.6b-v3"
PK_PUBLISHED_RTFX = 5.0      # README.md:151: Parakeet V3 "~5x real-time speed", CPU (i5), ONNX int8


def metric_for(model: str) -> str:
    name = model.split(":", 1)[-1].split(":")[0]
    return f"RTFx (audio-sec/wall-sec) Whisper-{name} 30s chunks @1/2/4/8 MI355X"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=8, help="30 s chunks per GPU")
    ap.add_argument("--model", default=MODEL_SPEC)
    ap.add_argument("--dtype", default="bf16")
    ap.add_argument("--decode-steps", type=int, default=N_STEPS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-app-latency", action="store_true", help="skip the B=1 whisper_full (app default) latency")
    ap.add_argument("--no-probe", action="store_true", help="skip the per-kernel HIP-event probes")
    ap.add_argument("--no-turbo", action="store_true", help="skip the Whisper Turbo (4 decoder layers) line")
    ap.add_argument("--no-c2", action="store_true", help="skip the Whisper-small f32 B=1 line (BASELINE config 2)")
    ap.add_argument("--no-parakeet", action="store_true", help="skip the Parakeet-V3 (BASELINE config 5) lines")
    ap.add_argument("--parakeet-only", action="store_true", help="only the Parakeet-V3 lines (developer runs)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL) for the real run; gloo only to rehearse N > 1 ranks on one GPU")
    ap.add_argument("--no-weight-bcast", action="store_true",
                    help="N > 1: every rank loads the model itself instead of rank 0 + RCCL broadcast")
    return ap.parse_args()


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(args) -> int:
    """Start args.gpus ranks of this script with torch.distributed.run (one process per GPU) as
    a child process; nothing in this process has touched the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")  # the CPU-baseline leg sets its own thread count
    return subprocess.call(cmd, env=env)


def host_cpu() -> dict:
    """CPU model and core counts of this host (the box's share is what the process may use)."""
    model, phys = None, set()
    try:
        cur = {}
        for line in open("/proc/cpuinfo"):
            if ":" not in line:
                if cur:
                    phys.add((cur.get("physical id"), cur.get("core id")))
                cur = {}
                continue
            k, v = (x.strip() for x in line.split(":", 1))
            cur[k] = v
            if k == "model name" and model is None:
                model = v
        if cur:
            phys.add((cur.get("physical id"), cur.get("core id")))
    except OSError:
        pass
    try:
        allowed = len(os.sched_getaffinity(0))
    except AttributeError:
        allowed = os.cpu_count()
    quota = None  # cgroup v2 CPU quota (the job's share of a shared host), in whole CPUs
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = max(1, int(int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return {"model": model, "physical_cores": len(phys) or None, "logical_cpus": os.cpu_count(),
            "affinity_cpus": allowed, "cgroup_cpu_quota": quota}


def cpu_threads(cpu: dict) -> int:
    """Threads for a CPU-baseline leg: every physical core this process may use, i.e.
    min(affinity CPUs, physical cores, cgroup CPU quota); an explicit
    SPT_CPU_THREADS overrides it."""
    if os.environ.get("SPT_CPU_THREADS"):
        return int(os.environ["SPT_CPU_THREADS"])
    n = [v for v in (cpu["affinity_cpus"], cpu["physical_cores"], cpu["cgroup_cpu_quota"]) if v]
    return max(1, min(n)) if n else 1


def cpu_baseline(model_spec: str, decode_steps: int) -> dict:
    """CPU baseline leg: the oracle (C restatement of the whisper-rs/whisper.cpp CPU path, fp32,
    OpenMP over this job's CPU share) on one 30 s chunk of the same workload, end to end:
    log-mel + encoder + cross K/V + the 4-token prompt pass + every decoder pass (no
    extrapolation).  The GPU box gives a one-GPU job 16 host cores (OMP_NUM_THREADS=16)."""
    from oracle import oracle as O
    name = model_spec.split(":")[1]
    cpu = host_cpu()
    threads = cpu_threads(cpu)
    O.set_threads(threads)
    dims = O.dims_for(name)
    m = O.Model(dims, 1234, O.W_F32)
    x = O.synth_audio(0)
    prompt = O.default_prompt(dims.n_vocab)
    t0 = time.perf_counter()
    mel = O.mel(x, dims.n_mels)
    t1 = time.perf_counter()
    enc = m.encode(mel)
    t2 = time.perf_counter()
    m.decode(enc, prompt, decode_steps, O.SUPPRESS_BLANK | O.NO_TIMESTAMPS | O.IGNORE_EOT)
    t3 = time.perf_counter()
    m.close()
    total = t3 - t0
    return {"value": round(CHUNK_S / total, 4), "unit": "audio-sec/wall-sec", "cores": threads, "kind": "port",
            "cpu_model": cpu["model"], "host_physical_cores": cpu["physical_cores"],
            "affinity_cpus": cpu["affinity_cpus"], "cgroup_cpu_quota": cpu["cgroup_cpu_quota"],
            "sample": f"1 x 30 s chunk, {name} dims fp32, {threads} OpenMP threads: mel {t1 - t0:.2f}s + encoder "
                      f"{t2 - t1:.2f}s + cross-KV + {PROMPT_LEN}-token prompt pass + {decode_steps - 1} decoder passes "
                      f"{t3 - t2:.2f}s = {total:.1f}s per chunk (timed whole, no extrapolation)"}


DOMINANT = "dec_cross_attn"  # largest share of device time (profiles/*_kernel_stats.csv)
# the kernels probed in situ with HIP events (spt_probe_kernel).  Only the dominant one is reported:
# r6 checked every probe against rocprofv3 over the same run (profiles/r6/probe_vs_rocprof_r6l.txt):
# the decoder cross-attention agrees within 1 %, while the other decoder probes read 5-8 % off and the
# encoder ones -1 % (fc1) and -9 % (attention: layer 0 repeated on the final residual rows is not the
# encoder's data, and the attention's running-maximum re-basing is data dependent), so per-kernel
# times of everything else come from the committed rocprofv3 summaries (profiles/r6/)
KERNEL_NAMES = {
    "dec_cross_attn": "cross_attn_kernel (decoder cross-attention, 1 layer)",
}


def roofline(eng, iters: int = 50):
    """Dominant-kernel roofline from HIP events on the engine's streams (spt_probe_kernel, on the
    buffers of the last timed call, in situ: the decoder cross-attention inside eager one-token
    passes over all layers with an event pair around it in each layer).
    achieved = algorithmic bytes (or flops) per launch / average launch duration.
    traffic = PMC-measured HBM bytes per launch of the same kernel, from the committed
    rocprofv3 --pmc summary (profiles/pmc_<kernel>.json), when present."""
    rows = {}
    for k, name in KERNEL_NAMES.items():
        p = eng.probe(k, iters)
        if p["work_is_flops"]:
            ach, peak, unit = p["work"] / p["avg_us"] / 1e6, MFMA_PEAK_BF16_TFS, "TFLOP/s"
        else:
            ach, peak, unit = p["work"] / p["avg_us"] / 1e3, HBM_PEAK_GBS, "GB/s"
        rows[k] = {"kernel": name, "bound": "mfma" if p["work_is_flops"] else "hbm", "avg_us": round(p["avg_us"], 3),
                   "work_per_launch": p["work"], "achieved": round(ach, 1), "peak": peak, "unit": unit,
                   "frac": round(ach / peak, 4)}
    dom = dict(rows[DOMINANT])
    traffic = None
    pmc = os.path.join(ROOT, "profiles", f"pmc_{DOMINANT}.json")
    if os.path.exists(pmc):
        traffic = json.load(open(pmc)).get("hbm_bytes_per_launch")
    roof = {"kernel": dom["kernel"], "bound": dom["bound"], "achieved": dom["achieved"], "peak": dom["peak"],
            "unit": dom["unit"], "frac": dom["frac"], "traffic": traffic, "avg_us": dom["avg_us"],
            "algorithmic_bytes_per_launch": dom["work_per_launch"]}
    return roof, rows


def phase_rooflines(info: dict, phases: dict, B: int, decode_steps: int, dtype: str) -> dict:
    """Whole-phase rooflines of the last call (HIP events per phase, engine stream):
    encoder = algorithmic FLOPs of conv stem + blocks / encoder time vs the dense
    MFMA peak of the dtype; decode pass = algorithmic bytes one greedy pass streams (layer
    weights + logits matrix + every sequence's cross K/V + self K/V at the mean position) /
    the mean pass time vs HBM peak."""
    d, L_e, L_d, V, nm = info["d"], info["n_enc"], info["n_dec"], info["n_vocab"], info["n_mels"]
    T, H = info["n_audio_ctx"], info["n_head"]
    esz = 2 if dtype == "bf16" else 4
    conv = 2 * 2 * T * d * 3 * nm + 2 * T * d * 3 * d
    layer = 2 * T * d * 3 * d + 4 * H * T * T * 64 + 2 * T * d * d + 2 * 2 * T * d * 4 * d
    enc_flops = B * (conv + L_e * layer)
    peak = MFMA_PEAK_BF16_TFS if dtype == "bf16" else FP32_PEAK_TFS
    out = {}
    if phases.get("encoder_ms", 0) > 0:
        tf = enc_flops / (phases["encoder_ms"] * 1e-3) / 1e12
        out["encoder"] = {"bound": "mfma", "flops_per_call": enc_flops, "ms": round(phases["encoder_ms"], 3),
                          "achieved": round(tf, 1), "peak": peak, "unit": "TFLOP/s", "frac": round(tf / peak, 4)}
    n_pass = phases.get("n_decode_passes", 0)
    if phases.get("decode_ms", 0) > 0 and n_pass > 1:
        mean_pos = PROMPT_LEN + (decode_steps - 1) / 2.0
        w = L_d * 14 * d * d * esz
        logit = V * d * esz
        cross = L_d * 2 * B * H * T * 64 * esz
        selfkv = L_d * 2 * B * H * mean_pos * 64 * esz
        per_pass = w + logit + cross + selfkv
        ms = phases["decode_ms"] / n_pass
        gbs = per_pass / (ms * 1e-3) / 1e9
        out["decode_pass"] = {"bound": "hbm", "bytes_per_pass": int(per_pass),
                              "bytes_split": {"layer_weights": w, "logits_matrix": logit, "cross_kv": cross,
                                              "self_kv_mean": int(selfkv)},
                              "ms_per_pass": round(ms, 4), "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(gbs / HBM_PEAK_GBS, 4)}
    return out


def parakeet_stage_work(info: dict, T: int, B: int) -> dict:
    """Algorithmic work of one Parakeet encoder pass over B utterances of T mel frames, per stage
    class of spt_parakeet_profile_encoder (SURVEY §8d style): (work, kind) with kind "f16"
    (MFMA flops), "f32" (f32 MFMA flops) or "hbm" (bytes).  Subsampling convolutions + linear;
    the relative-position projection once per pass (every layer's linear_pos over the 2 T3 - 1
    shared positions); the two half-FFNs, q/k/v/out and the convolution module's pointwise pair
    over the T3 frames; attention's q.k, q.p and p.v over the T3 x T3 pairs; the depthwise stage
    as its GLU input read + output write (f16); the LayerNorms as the residual rows they read and
    write: five per layer, four of them folding one pending f32 product and three writing x back
    (the split-K slabs beyond one product are the implementation's, not counted)."""
    h = lambda t: (t - 1) // 2 + 1
    d, ff, C, L, P, K = info["d"], info["ff"], info["sub_ch"], info["n_layers"], info["pred"], info["conv_k"]
    T1, T2, T3 = h(T), h(h(T)), h(h(h(T)))
    F1, F2, F3 = h(info["n_mels"]), h(h(info["n_mels"])), h(h(h(info["n_mels"])))
    rows = B * T3
    sub = 2 * 9 * C * T1 * F1 + 2 * 9 * C * (T2 * F2 + T3 * F3) + 2 * C * C * (T2 * F2 + T3 * F3) + 2 * C * F3 * d * T3
    return {"subsampling": (B * sub, "f16"),
            "pos": (2 * (2 * T3 - 1) * d * d * L, "f16"),
            "layernorm": (rows * L * 60 * d, "hbm"),
            "ffn": (rows * L * 8 * d * ff, "f16"),
            "qkv_out": (rows * L * 8 * d * d, "f16"),
            "attn": (B * L * 6 * T3 * T3 * d, "f16"),
            "conv_pw": (rows * L * 6 * d * d, "f16"),
            "conv_dw": (rows * L * 6 * d, "hbm"),
            "joint_enc": (rows * 2 * d * P, "f32")}


def parakeet_encoder_flops(info: dict, T: int, B: int) -> int:
    """Algorithmic FLOPs of one Parakeet encoder pass over B utterances of T mel frames: the MFMA
    stages of parakeet_stage_work (the depthwise convolution's 2 K flops per element aside)."""
    return int(sum(w for w, k in parakeet_stage_work(info, T, B).values() if k != "hbm"))


def parakeet_kernels(e, info: dict, T: int, B: int, iters: int = 3) -> dict:
    """Per-stage rooflines of the last call's encoder pass: spt_parakeet_profile_encoder re-runs it
    eagerly (same buffers, bitwise the same output) with a HIP event after every stage; ms per
    pass per stage class vs that stage's algorithmic work (parakeet_stage_work)."""
    ms = e.profile_encoder(iters)
    out = {}
    for k, (w, kind) in parakeet_stage_work(info, T, B).items():
        t = ms[k]
        if kind == "hbm":
            ach, peak, unit = w / (t * 1e-3) / 1e9 if t > 0 else 0.0, HBM_PEAK_GBS, "GB/s"
        else:
            ach, peak, unit = w / (t * 1e-3) / 1e12 if t > 0 else 0.0, (FP32_PEAK_TFS if kind == "f32" else MFMA_PEAK_F16_TFS), "TFLOP/s"
        out[k] = {"ms": round(t, 4), "work": int(w), "bound": "hbm" if kind == "hbm" else "mfma", "achieved": round(ach, 1),
                  "peak": peak, "unit": unit, "frac": round(ach / peak, 4)}
    out["sum_ms"] = round(sum(ms.values()), 4)
    return out


def parakeet_bench(device: int, steps: int, warmup: int, with_cpu: bool) -> dict:
    """BASELINE config 5 (BASELINE.json configs[4]): Parakeet-V3 -- synthetic
    parakeet-tdt-0.6b-v3 weights (NeMo FastConformer-TDT shape, 24 layers, d 1024), fp16 encoder,
    f32 TDT greedy decoding, the app's Segment timestamps, host PCM in, text out.
      * streaming: 64 concurrent 1 s windows per pass (RTFx = 64 s / pass wall time), and one
        1 s window alone (the latency of a single stream's window);
      * offline: 8 x 30 s chunks per pass (the app's whole-recording call, batched).
    cpu_baseline: the oracle (C restatement, fp32, OpenMP) end to end on 20 of the streaming line's
    own 1 s windows, one at a time."""
    import numpy as np
    from spittle_amd import ParakeetEngine, ParakeetInferenceParams, ParakeetModelParams, TimestampGranularity
    from spittle_amd.synth import synth_audio
    e = ParakeetEngine()
    e.load_model_with_params(PK_SPEC, ParakeetModelParams(dtype="f16", device=device, max_batch=64, max_seconds=30.0))
    info = e.info()
    prm = ParakeetInferenceParams(timestamp_granularity=TimestampGranularity.Segment)

    def run(batch):
        for _ in range(warmup):
            e.transcribe_batch(batch, prm)
        ts, res = [], None
        for _ in range(steps):
            t0 = time.perf_counter()
            res = e.transcribe_batch(batch, prm)
            ts.append(time.perf_counter() - t0)
        return float(np.median(ts)), float(np.sum(ts)), res, e.timings()

    out = {"model": PK_SPEC, "dtype": "f16 encoder, f32 prediction network + joint",
           "data": "synthetic (BASELINE.md §3 seeded 16 kHz signal; random-init weights)"}
    only = os.environ.get("PK_BENCH_ONLY", "")  # developer profiling: one workload
    w1 = [synth_audio(3000 + i)[:16000] for i in range(64)]
    if only == "offline":
        w1 = w1[:1]
    med, tot, res, ph = run(w1)
    flops = parakeet_encoder_flops(info, 16000 // 160, len(w1))
    tf = flops / (ph["encoder_ms"] * 1e-3) / 1e12
    out["streaming_1s_b64"] = {"rtfx": round(64 * steps / tot, 2), "ms_per_pass_median": round(med * 1e3, 3),
                               "phases_ms": {k: round(v, 3) for k, v in ph.items() if k.endswith("_ms")},
                               "decode_steps": ph["n_steps"], "tokens_first_window": len(res[0].tokens),
                               "encoder_roofline": {"bound": "mfma", "flops_per_call": flops, "achieved": round(tf, 1),
                                                    "peak": MFMA_PEAK_F16_TFS, "unit": "TFLOP/s",
                                                    "frac": round(tf / MFMA_PEAK_F16_TFS, 4)},
                               "kernels": parakeet_kernels(e, info, 16000 // 160, len(w1))}
    if only == "stream64":
        e.unload_model()
        return out
    med, tot, res, ph = run(w1[:1])
    out["streaming_1s_b1_latency_ms"] = {"median": round(med * 1e3, 3),
                                         "phases_ms": {k: round(v, 3) for k, v in ph.items() if k.endswith("_ms")},
                                         "decode_steps": ph["n_steps"]}
    w30 = [synth_audio(i) for i in range(8)]
    if only == "stream":
        w30 = [w30[0][:16000]]
    med, tot, res, ph = run(w30)
    flops = parakeet_encoder_flops(info, 480000 // 160, len(w30))
    tf = flops / (ph["encoder_ms"] * 1e-3) / 1e12
    out["offline_30s_b8"] = {"rtfx": round(8 * 30.0 * steps / tot, 2), "ms_per_pass_median": round(med * 1e3, 3),
                             "phases_ms": {k: round(v, 3) for k, v in ph.items() if k.endswith("_ms")},
                             "decode_steps": ph["n_steps"], "tokens_first_chunk": len(res[0].tokens),
                             "encoder_roofline": {"bound": "mfma", "flops_per_call": flops, "achieved": round(tf, 1),
                                                  "peak": MFMA_PEAK_F16_TFS, "unit": "TFLOP/s",
                                                  "frac": round(tf / MFMA_PEAK_F16_TFS, 4)},
                             "kernels": parakeet_kernels(e, info, 480000 // 160, len(w30))}
    out["vs_published_cpu_rtfx"] = {"published": PK_PUBLISHED_RTFX, "source": "README.md:151 (i5 CPU, ONNX int8)",
                                    "streaming_ratio": round(out["streaming_1s_b64"]["rtfx"] / PK_PUBLISHED_RTFX, 1)}
    e.unload_model()
    if with_cpu:
        from oracle import parakeet as PO
        cpu = host_cpu()
        threads = cpu_threads(cpu)
        PO.set_threads(threads)
        m = PO.Model(PO.dims_for("parakeet-tdt-0.6b-v3"), 1234, PO.W_F32)
        # the streaming line's own windows (the first 20 of its 64 x 1 s windows), one at a time
        nw = min(20, len(w1))
        t0 = time.perf_counter()
        for x in w1[:nw]:
            m.decode(m.encode(PO.mel(x)))
        dt = time.perf_counter() - t0
        m.close()
        out["cpu_baseline"] = {"value": round(float(nw) / dt, 3), "unit": "audio-sec/wall-sec", "cores": threads,
                               "kind": "port", "cpu_model": cpu["model"], "affinity_cpus": cpu["affinity_cpus"],
                               "sample": f"{nw} of streaming_1s_b64's 1 s windows (synth_audio(3000..{3000 + nw - 1})), "
                                         f"one at a time, parakeet-tdt-0.6b-v3 dims fp32, {threads} OpenMP threads, "
                                         f"mel + encoder + TDT greedy {dt:.2f}s (timed whole)"}
    return out


def resampler_bench(device: int, with_cpu: bool) -> dict:
    """Capture-side resampler (ABI 7): one 48 kHz capture stream per call (8 x 30 s
    concatenated, host buffer in, 16 kHz frames out), FrameResampler::new + push(all) + finish.
    Roofline: the unit GEMM's f32 MFMA FLOPs (2 * Kp * Np per rubato unit) over the call time."""
    import numpy as np
    from spittle_amd.resampler import FrameResampler
    fin, secs = 48000, 240.0
    rng = np.random.default_rng(1000)
    x = np.clip(0.1 * rng.standard_normal(int(fin * secs)), -1, 1).astype(np.float32)
    r = FrameResampler(fin, 16000, 0.030, device)
    nin, nout = r.fft_sizes
    for _ in range(2):
        r.process_stream(x)
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        r.process_stream(x)
        ts.append(time.perf_counter() - t0)
    t = sorted(ts)[len(ts) // 2]
    units = (-(-len(x) // 1024) * 1024) // nin
    kp, np_ = -(-nin // 32) * 32, -(-(2 * nout) // 128) * 128
    flops = 2.0 * units * kp * np_
    out = {"workload": f"one {secs:.0f} s 48 kHz stream -> 16 kHz 30 ms frames (rubato FftFixedIn units {nin}->{nout})",
           "rtfx": round(secs / t, 1), "ms_per_call_median": round(t * 1e3, 3),
           "gemm_roofline": {"bound": "mfma", "flops_per_call": flops, "achieved_tflops_whole_call": round(flops / t / 1e12, 2),
                             "peak": 157.3, "unit": "TFLOP/s", "note": "whole call incl. H2D/D2H of the host buffers"}}
    if with_cpu:
        from oracle import resampler as R
        xs = x[: fin * 30].astype(np.float64)
        t0 = time.perf_counter()
        R.resample_fast(xs, fin, 16000)
        tc = time.perf_counter() - t0
        out["cpu_baseline"] = {"value": round(30.0 / tc, 1), "unit": "audio-sec/wall-sec", "cores": 1, "kind": "port",
                               "sample": "30 s of the same stream, numpy restatement of FftFixedIn (f64, block-parallel)"}
    r.close()
    return out


def _stats_fields(eng, ms: float) -> dict:
    """The call's engine runs and decoder passes (spt_get_call_stats) beside its wall time."""
    cs = eng.call_stats()
    n = max(1, cs["decoder_passes"])
    return {"ms": round(ms, 2), "engine_calls": cs["engine_calls"], "encoder_windows": cs["encoder_windows"],
            "decoder_passes": cs["decoder_passes"],
            "device_ms": round(cs["device_ms"], 2), "encoder_ms": round(cs["encoder_ms"], 2),
            "decode_ms": round(cs["decode_ms"], 2), "decode_ms_per_pass": round(cs["decode_ms"] / n, 4),
            "host_ms": round(ms - cs["device_ms"], 2)}


def app_latency(eng, info: dict, dtype: str, dur_s=(5, 10, 30)) -> dict:
    """The app's real call (transcription.rs:494-503): one utterance (B = 1), whisper_full with
    its default parameters (timestamps on, temperature fallback 0.2 / best_of 5), language
    "en", through spt_transcribe.  Random-init weights never emit EOT or confident tokens, so
    every window decodes to its token limit and falls back through every temperature: an
    upper bound of the app's latency.  Each case reports its decoder runs (engine_calls: one per
    window and temperature), its encoder runs (encoder_windows: one per window, shared by every
    temperature and decoder since ABI 11), decoder passes and the device time behind them
    (spt_get_call_stats);
    decode_ms_per_pass mixes 1-row greedy passes and 5-row (best_of) sampled passes.
    `b1_greedy_pass` isolates the B = 1 pass: one 30 s window on the greedy fast path, its mean
    decoder pass against the bytes that pass streams (every layer weight, the logits matrix, one
    utterance's cross K/V and its self K/V at the mean position)."""
    from spittle_amd import WhisperInferenceParams
    from spittle_amd.synth import synth_audio
    out = {}
    p = WhisperInferenceParams(language="en")
    eng.transcribe_samples(synth_audio(2000)[:16000 * 5], p)  # warm (graphs captured)
    for s in dur_s:
        x = synth_audio(2000 + s)[:16000 * s]
        t0 = time.perf_counter()
        r = eng.transcribe_samples(x, p)
        ms = (time.perf_counter() - t0) * 1e3
        out[f"{s}s"] = dict(_stats_fields(eng, ms), windows=r.n_windows, fallbacks=r.n_fallbacks,
                            tokens=len(r.tokens), segments=len(r.segments))
    # beam search (whisper.cpp's WHISPER_SAMPLING_BEAM_SEARCH, beam_size 5; one captured graph per
    # step, the candidate bookkeeping on the host), 10 s, no fallback
    pb = WhisperInferenceParams(language="en", beam_size=5, temperature_inc=0.0)
    x = synth_audio(2010)[:16000 * 10]
    eng.transcribe_samples(x, pb)  # warm: the step graph is captured on first use
    t0 = time.perf_counter()
    r = eng.transcribe_samples(x, pb)
    ms = (time.perf_counter() - t0) * 1e3
    st = _stats_fields(eng, ms)
    cs = eng.call_stats()
    out["10s_beam5"] = dict(st, windows=r.n_windows, tokens=len(r.tokens), beam_steps=cs["beam_steps"],
                            ms_per_decoder_step=round(ms / max(1, cs["decoder_passes"]), 3))
    # the B = 1 decoder pass alone (fast path, 30 s, 128 steps)
    pg = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                                max_new_tokens=N_STEPS)
    x = synth_audio(2030)
    eng.transcribe_samples(x, pg)
    t0 = time.perf_counter()
    eng.transcribe_samples(x, pg)
    ms = (time.perf_counter() - t0) * 1e3
    roof = phase_rooflines(info, eng.timings(), 1, N_STEPS, dtype).get("decode_pass", {})
    out["b1_greedy_pass"] = dict(_stats_fields(eng, ms), bytes_per_pass=roof.get("bytes_per_pass"),
                                 ms_per_pass=roof.get("ms_per_pass"), achieved_GBs=roof.get("achieved"),
                                 frac_of_hbm_peak=roof.get("frac"))
    return out


def turbo_bench(device: int, pcm_list, steps: int, warmup: int, decode_steps: int) -> dict:
    """The catalog's Whisper Turbo (ggml-large-v3-turbo.bin: model_catalog.json:169-173) on the
    same protocol and batch: large-v3's 32-layer encoder with 4 decoder layers (synthetic weights,
    synthetic:large-v3:dec=4).  RTFx of the median step, phase times, decoder pass time."""
    import numpy as np
    from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
    B = len(pcm_list)
    e = WhisperEngine(WhisperModelParams(dtype="bf16", device=device, max_batch=B, seed=1234))
    e.load_model("synthetic:large-v3:dec=4")
    p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                               max_new_tokens=decode_steps)
    for _ in range(warmup):
        e.transcribe_batch(pcm_list, p)
    marks = [time.perf_counter()]
    for _ in range(steps):
        e.transcribe_batch(pcm_list, p)
        marks.append(time.perf_counter())
    med = float(np.median(np.diff(marks)))
    t = e.timings()
    e.unload_model()
    return {"model": "synthetic:large-v3:dec=4 (ggml-large-v3-turbo geometry: 32 encoder + 4 decoder layers)",
            "batch": B, "steps": steps, "rtfx": round(B * CHUNK_S / med, 2), "ms_per_step": round(med * 1e3, 3),
            "phases_ms": {k: round(v, 3) for k, v in t.items() if k.endswith("_ms")},
            "decode_ms_per_pass": round(t["decode_ms"] / max(1, t["n_decode_passes"]), 4)}


C2_SPEC = "synthetic:small"
C2_TRAFFIC_JSON = "profiles/r6/pmc_c2_small_f32.json"


def small_f32_bench(device: int, steps: int, warmup: int, decode_steps: int, with_cpu: bool) -> dict:
    """BASELINE.json configs[1] (C2): Whisper-small, fp32 end to end (exact-f32 MFMA), one 30 s
    chunk per call (B = 1: the app's one-utterance call, transcription.rs:494-503), the benchmark
    protocol (greedy en, no timestamps, 4-token prompt + decode_steps passes, EOT ignored), host PCM
    in, text out.  RTFx of the median call; encoder fraction of the 157.3 TF f32 peak; decode-pass
    HBM fraction (bytes one pass streams / mean pass time); `traffic`: PMC FETCH_SIZE of the C2
    decode pass's kernels per pass from its own rocprofv3 run (scripts/c2_pmc.sh ->
    profiles/r6/pmc_c2_small_f32.json), never the large-v3 figure; cpu_baseline: the oracle on
    the same chunk, whole (mel + encoder + every decoder pass)."""
    import numpy as np
    from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
    from spittle_amd.synth import synth_audio
    e = WhisperEngine(WhisperModelParams(dtype="f32", device=device, max_batch=1, seed=1234))
    e.load_model(C2_SPEC)
    info = e.info()
    p = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                               max_new_tokens=decode_steps)
    x = synth_audio(0)
    for _ in range(warmup):
        e.transcribe_samples(x, p)
    marks = [time.perf_counter()]
    for _ in range(steps):
        r = e.transcribe_samples(x, p)
        marks.append(time.perf_counter())
    assert len(r.tokens) == decode_steps
    med = float(np.median(np.diff(marks)))
    t = e.timings()
    roofs = phase_rooflines(info, t, 1, decode_steps, "f32")
    e.unload_model()
    dp = roofs.get("decode_pass", {})
    if dp:
        dp["traffic"] = None
        pmc = os.path.join(ROOT, C2_TRAFFIC_JSON)
        if os.path.exists(pmc):
            j = json.load(open(pmc))
            dp["traffic"] = j.get("hbm_bytes_per_pass")
            dp["traffic_ratio"] = round(j["hbm_bytes_per_pass"] / dp["bytes_per_pass"], 3)
            dp["traffic_source"] = C2_TRAFFIC_JSON
    out = {"model": C2_SPEC, "dtype": "f32", "batch": 1, "steps": steps, "rtfx": round(CHUNK_S / med, 2),
           "ms_per_call_median": round(med * 1e3, 3),
           "phases_ms": {k: round(v, 3) for k, v in t.items() if k.endswith("_ms")},
           "rooflines": roofs}
    if with_cpu:
        out["cpu_baseline"] = cpu_baseline(C2_SPEC, decode_steps)
    return out


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if args.gpus > 1 and world_env is None:
        sys.exit(launch_ranks(args))
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(world_env or "1")
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    if world > 1:
        local %= max(1, torch.cuda.device_count())  # rehearsal: several ranks on one GPU (gloo)
        torch.cuda.set_device(local)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.dist_backend)
        assert dist.get_world_size() == args.gpus
    dev = torch.device("cuda", local)
    if args.parakeet_only:
        torch.cuda.synchronize()
        print(json.dumps({"parakeet": parakeet_bench(local, args.steps, args.warmup, not args.no_cpu_baseline)}),
              flush=True)
        return

    from spittle_amd import WhisperEngine, WhisperInferenceParams, WhisperModelParams
    from spittle_amd.dist import broadcast_weights, max_over_ranks, shard_range
    from spittle_amd.synth import synth_audio

    B = args.batch
    # this rank's shard of the global utterance list (B per GPU: weak scaling)
    lo, hi = shard_range(world * B, world, rank)
    pcm = np.stack([synth_audio(i) for i in range(lo, hi)])
    pcm_list = [pcm[i] for i in range(B)]
    pcm_dev = torch.from_numpy(pcm).to(dev)
    torch.cuda.synchronize()

    # N > 1: rank 0 loads (generates / dequantises) the weights, one RCCL broadcast over xGMI
    # writes its arena into the other ranks' engines; outside the timed region
    bcast = world > 1 and not args.no_weight_bcast
    eng = WhisperEngine(WhisperModelParams(dtype=args.dtype, device=local, max_batch=B, seed=1234,
                                           external_weights=bcast and rank != 0))
    t_load = time.perf_counter()
    eng.load_model(args.model)
    load_ms = (time.perf_counter() - t_load) * 1e3
    wload = None
    if bcast:
        bi = broadcast_weights(eng, device=dev)
        bms = max_over_ranks(bi["ms"], device=dev)
        wload = {"mode": "rank 0 load + " + ("RCCL" if args.dist_backend == "nccl" else args.dist_backend) +
                 " broadcast into the arenas (" + bi.get("path", "") + ")", "bytes": bi["bytes"], "ms": round(bms, 3),
                 "GB/s": round(bi["bytes"] / bms / 1e6, 1) if bms > 0 else None,
                 "rank0_load_ms": round(max_over_ranks(load_ms if rank == 0 else 0.0, device=dev), 1)}
    info = eng.info()
    params = WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True,
                                    max_new_tokens=args.decode_steps)
    lens = [pcm.shape[1]] * B

    def step_host():  # BASELINE.md:48: host PCM buffer -> text on the host
        return eng.transcribe_batch(pcm_list, params)

    def step_dev():
        return eng.transcribe_batch_device(pcm_dev.data_ptr(), pcm.shape[1], lens, params)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    def timed(step):
        for _ in range(args.warmup):
            step()
        barrier()
        t0 = time.perf_counter()
        marks = [t0]
        res = None
        for _ in range(args.steps):
            res = step()  # returns host tokens and text: each step ends synchronised
            marks.append(time.perf_counter())
        barrier()
        dt = max_over_ranks(time.perf_counter() - t0, device=dev)
        assert all(len(r.tokens) == args.decode_steps for r in res)
        return dt, float(np.median(np.diff(marks))), eng.timings()

    dt, med, phases = timed(step_host)
    dt_dev, med_dev, phases_dev = timed(step_dev)
    rank_ms = [None] * world
    if world > 1:
        dist.all_gather_object(rank_ms, round(med * 1e3, 3))
    # the median step; the slowest rank's median (weak scaling: every rank's
    # step must finish), next to the mean over the barrier-bracketed region
    med_max = max_over_ranks(med, device=dev)
    med_dev_max = max_over_ranks(med_dev, device=dev)

    audio_step = world * B * CHUNK_S
    value = audio_step / med_max
    value_mean = audio_step * args.steps / dt
    ms_per_step = med_max * 1000.0

    roof = kernels = None
    cpu = app = None
    if rank == 0:
        if not args.no_probe:
            roof, kernels = roofline(eng)
        if world == 1 and not args.no_app_latency:
            app = app_latency(eng, info, args.dtype)
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.model, args.decode_steps)
    rs = None
    if rank == 0 and world == 1 and not args.no_parakeet:
        rs = resampler_bench(local, not args.no_cpu_baseline)
    tb = None
    if rank == 0 and world == 1 and not args.no_turbo and args.model == "synthetic:large-v3":
        tb = turbo_bench(local, pcm_list, min(args.steps, 5), 1, args.decode_steps)
    c2 = None
    if rank == 0 and world == 1 and not args.no_c2 and args.model == "synthetic:large-v3":
        c2 = small_f32_bench(local, args.steps, args.warmup, args.decode_steps, not args.no_cpu_baseline)
    pk = None
    if rank == 0 and world == 1 and not args.no_parakeet:
        eng.unload_model()  # free the Whisper arenas first
        pk = parakeet_bench(local, min(args.steps, 10), max(1, args.warmup), not args.no_cpu_baseline)
    if rank == 0:
        out = {
            "metric": metric_for(args.model), "value": round(value, 3), "unit": "audio-sec/wall-sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(ms_per_step, 3),
            "value_stat": "median step (max over ranks)", "value_mean": round(value_mean, 3),
            "ms_per_step_mean": round(dt * 1000.0 / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": args.dtype,
            "data": f"synthetic (BASELINE.md §3 seeded 16 kHz signal; random-init {args.model.split(':', 1)[-1]} weights)",
            "config": {"workload": f"whisper-{args.model.split(':')[-1]} 30s chunks, batch {B}/GPU, greedy en, "
                                   f"{PROMPT_LEN}-token prompt + {args.decode_steps} decode steps, host PCM in, text out",
                       "model": args.model, "global_batch": world * B, "seq_len": 1500,
                       "decode_steps": args.decode_steps, "parallelism": f"replicas x{world} (utterance shards)"},
            "value_device_resident": round(audio_step / med_dev_max, 3),
            "ms_per_step_device_resident": round(med_dev_max * 1000.0, 3),
            "phases_ms": {k: round(v, 3) for k, v in phases.items() if k.endswith("_ms")},
            "phases_ms_device_resident": {k: round(v, 3) for k, v in phases_dev.items() if k.endswith("_ms")},
            "roofline": roof, "rooflines": phase_rooflines(info, phases, B, args.decode_steps, args.dtype),
            "kernels": kernels, "cpu_baseline": cpu,
        }
        if app:
            out["app_call_latency_b1"] = app
        if world > 1:
            out["ms_per_step_per_rank"] = rank_ms
        if wload:
            out["weight_load"] = wload
        if tb:
            out["whisper_turbo"] = tb
        if c2:
            out["whisper_small_f32_b1"] = c2
        if pk:
            out["parakeet_v3"] = pk
        if rs:
            out["resampler"] = rs
        print(json.dumps(out), flush=True)
    eng.unload_model()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
