"""GPU checks of the multi-GPU plumbing that one MI355X can exercise:

* the weight arena seen from torch aliases the engine's (the broadcast target), and a context
  created with external weights transcribes bit-identically once rank 0's bytes are written
  into it and committed;
* spt_ctx_create_replicas / spt_transcribe_batch_replicas (one host process over a device list)
  with the single device of this box;
* bench.py --gpus 2 launches its own two ranks (gloo rehearsal on one GPU) and reports them;
* batches whose prompt rows exceed 64 (max_batch 17: 17 x 4 prompt rows) decode like smaller ones.
"""
import ctypes as C
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _params(**kw):
    from spittle_amd import WhisperInferenceParams
    kw.setdefault("max_new_tokens", 8)
    return WhisperInferenceParams(language="en", no_timestamps=True, temperature_inc=0.0, ignore_eot=True, **kw)


def test_arena_alias_and_external_commit():
    import torch
    from spittle_amd import WhisperEngine, WhisperModelParams
    from spittle_amd.dist import arena_tensor
    src = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=2, seed=77))
    src.load_model("synthetic:tiny")
    dst = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=2, seed=77, external_weights=True))
    dst.load_model("synthetic:tiny")
    a, b = arena_tensor(src, "cuda:0"), arena_tensor(dst, "cuda:0")
    assert a.data_ptr() == src.weights_arena()[0] and a.numel() == src.info()["weight_bytes"]
    # the exported bytes are the aliased bytes
    ref = torch.empty_like(a)
    src.export_weights(ref.data_ptr(), ref.numel())
    assert torch.equal(ref, a)
    x = [O.synth_audio(5)]
    with pytest.raises(Exception, match="weights not loaded"):
        dst.transcribe_batch(x, _params())
    b.copy_(a)  # what the broadcast does on a receiving rank
    dst.commit_weights()
    r1, r2 = src.transcribe_batch(x, _params())[0], dst.transcribe_batch(x, _params())[0]
    assert r1.tokens == r2.tokens and np.array_equal(r1.top1, r2.top1)
    src.unload_model()
    dst.unload_model()


def test_replicas_api_single_device():
    from spittle_amd import _lib as L
    from spittle_amd.engine import WhisperEngine, WhisperModelParams, _infer_params, _take_result
    lib = L.load()
    mp = L.ModelParams()
    lib.spt_default_model_params(C.byref(mp))
    mp.max_batch = 2
    devs = (C.c_int32 * 1)(0)
    ctxs = (C.c_void_p * 1)()
    ms = C.c_double(-1.0)
    err = C.create_string_buffer(512)
    st = lib.spt_ctx_create_replicas(b"synthetic:tiny", C.byref(mp), devs, 1, ctxs, C.byref(ms), err, 512)
    assert st == L.SPT_OK, err.value
    assert ms.value == 0.0
    dup = (C.c_int32 * 2)(0, 0)
    two = (C.c_void_p * 2)()
    assert lib.spt_ctx_create_replicas(b"synthetic:tiny", C.byref(mp), dup, 2, two, None, err, 512) == L.SPT_ERR_INVALID_ARG
    xs = [np.ascontiguousarray(O.synth_audio(30 + i, n), np.float32) for i, n in enumerate([480000, 100000, 0])]
    keep = []
    ip = _infer_params(_params(), keep)
    fp = C.POINTER(C.c_float)
    ptrs = (fp * 3)(*[x.ctypes.data_as(fp) for x in xs])
    lens = (C.c_size_t * 3)(*[x.size for x in xs])
    out = (C.POINTER(L.Result) * 3)()
    assert lib.spt_transcribe_batch_replicas(ctxs, 1, ptrs, lens, 3, C.byref(ip), out) == L.SPT_OK
    got = [_take_result(out[i]) for i in range(3)]
    lib.spt_ctx_destroy(ctxs[0])
    ref = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=2, seed=1234))
    ref.load_model("synthetic:tiny")
    want = ref.transcribe_batch(xs, _params())
    ref.unload_model()
    for g, w in zip(got, want):
        assert g.tokens == w.tokens and g.text == w.text
    assert got[2].text == "" and got[2].tokens == []


@pytest.mark.parametrize("max_batch", [16, 17])
def test_prompt_rows_over_64(max_batch):
    """17 sequences x 4 prompt tokens = 68 decoder rows: the prompt is prefilled in chunks and
    the logits pass runs on its last token; every window equals its batch-of-one result, bitwise
    (a row's arithmetic never depends on its neighbours: MFMA rows, per-(b, h) attention, per-row
    LayerNorm, and a chunked prefill attends to the same keys in the same order)."""
    from spittle_amd import WhisperEngine, WhisperModelParams
    e = WhisperEngine(WhisperModelParams(dtype="bf16", max_batch=max_batch, seed=1234))
    e.load_model("synthetic:tiny")
    xs = [O.synth_audio(40 + i, 32000) for i in range(max_batch)]
    p = _params()
    together = e.transcribe_batch(xs, p)
    for i in (0, max_batch - 1):
        alone = e.transcribe_samples(xs[i], p)
        assert alone.tokens == together[i].tokens
        np.testing.assert_array_equal(np.array(alone.top1), np.array(together[i].top1))
    e.unload_model()


def test_bench_launches_its_own_ranks(tmp_path):
    """`bench.py --gpus 2` (no WORLD_SIZE) starts two ranks itself; gloo lets both share this
    box's one GPU.  The line reports both ranks and the in-place weight broadcast."""
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dist-backend", "gloo",
           "--model", "synthetic:tiny", "--batch", "2", "--decode-steps", "8", "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--no-app-latency", "--no-probe"]
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["global_batch"] == 4
    assert len(line["ms_per_step_per_rank"]) == 2
    assert line["weight_load"]["bytes"] > 0
    assert line["value"] > 0
