"""``oneshot`` -- drop-in for the ``llmcompressor.oneshot`` call the reference makes at
scripts/do_oneshot.py:179-187, plus ``save_compressed`` for ``model.save_pretrained(...,
save_compressed=True)`` (scripts/do_oneshot.py:197).

Flow, one process per GPU:
  recipe -> modifiers -> per-module schemes (targets / ignore)
  [AWQ] layer-sequential calibration: capture layer-0 inputs, then per decoder layer:
        onload -> statistics + grid search + smoothing (awq.py) -> propagate outputs -> offload
  quantization state: every targeted weight gets its scheme; the compressed tensors are
        produced by the fused HIP kernel (ops.compress_weight) at save time or on demand.
The returned model keeps bf16 (smoothed) weights; ``model.quantization_scheme_map`` names the
scheme of each targeted module (same names as the reference's per-expert Linear layout).
"""
from __future__ import annotations

import logging
import os
import threading
import time
from typing import Any, Dict, Iterable, List, Optional, Tuple, Union

import torch
from torch import nn

from . import awq as awq_mod
from .dense_mlp import fused_mlps
from .dense_norm import fused_rmsnorms
from .rotary import fused_rotary
from .moe_eager import eager_experts
from .patching import bmm_guard
from .model import checkpoint_name, decoder_layers, iter_linears, model_type
from .quantization import QuantizationScheme
from .recipe import AWQModifier, QuantizationModifier, match_any, match_precedence, parse_recipe

log = logging.getLogger(__name__)


class _StopForward(Exception):
    pass


def resolve_schemes(model: nn.Module, modifiers: List[QuantizationModifier]) -> Dict[str, Tuple[QuantizationScheme, QuantizationModifier]]:
    """module name -> (scheme, owning modifier); later modifiers do not override earlier ones.
    Within a modifier, a module matched by several config groups takes the group of its most
    specific target, as compressed-tensors resolves overlapping targets: exact name, then
    ``re:`` regex, then class name (ties: the first group in recipe order)."""
    out: Dict[str, Tuple[QuantizationScheme, QuantizationModifier]] = {}
    refs = iter_linears(model)
    for mod in modifiers:
        for ref in refs:
            if ref.name in out:
                continue
            if match_any(ref.name, ref.type_name, mod.ignore):
                continue
            best = None
            for order, scheme in enumerate(mod.config_groups.values()):
                if scheme.weights is None:
                    continue
                ranks = [r for r in (match_precedence(ref.name, ref.type_name, t) for t in scheme.targets)
                         if r is not None]
                if ranks and (best is None or (min(ranks), order) < best[0]):
                    best = ((min(ranks), order), scheme)
            if best is not None:
                out[ref.name] = (best[1], mod)
    return out


def _batches(dataset, num_samples: Optional[int], max_seq_length: Optional[int], device) -> List[Dict[str, torch.Tensor]]:
    """Tokenized dataset (HF Dataset / list of dicts / tensor) -> list of batch-1 model inputs."""
    if dataset is None:
        return []
    rows: Iterable
    if torch.is_tensor(dataset):
        rows = [{"input_ids": r} for r in dataset]
    else:
        rows = dataset
    out = []
    for i, r in enumerate(rows):
        if num_samples is not None and i >= num_samples:
            break
        ids = r["input_ids"]
        ids = torch.as_tensor(ids, dtype=torch.long).reshape(1, -1)
        if max_seq_length:
            ids = ids[:, :max_seq_length]
        b = {"input_ids": ids.to(device)}
        if "attention_mask" in r and r["attention_mask"] is not None:
            b["attention_mask"] = torch.as_tensor(r["attention_mask"], dtype=torch.long).reshape(1, -1)[:, :ids.shape[1]].to(device)
        out.append(b)
    return out


@torch.no_grad()
def _capture_layer0_inputs(model: nn.Module, layers: nn.ModuleList, batches) -> List[Tuple[tuple, dict]]:
    cached: List[Tuple[tuple, dict]] = []

    def hook(mod, args, kwargs):
        kw = {k: v for k, v in kwargs.items() if k not in ("past_key_values", "past_key_value", "use_cache")}
        kw["use_cache"] = False
        cached.append((args, kw))
        raise _StopForward

    h = layers[0].register_forward_pre_hook(hook, with_kwargs=True)
    ts = []
    try:
        for b in batches:
            t0 = time.time()
            try:
                model(**b, use_cache=False)
            except _StopForward:
                pass
            if awq_mod.PHASE_TIMING:  # diagnostics: per-sample wall time, synchronised
                torch.cuda.synchronize()
                ts.append(round(time.time() - t0, 4))
    finally:
        h.remove()
    if ts:
        log.info("AWQ: layer-0 capture per sample (s, synchronised): %s", ts)
    return cached


def _layer_out(o):
    return o[0] if isinstance(o, tuple) else o


@torch.no_grad()
def _sequential_awq(model: nn.Module, awq: AWQModifier, schemes, batches, device, report,
                    calibrate_all_experts: bool = True, stateful_observers: bool = False, residency=None,
                    seconds: Optional[List[float]] = None, awq_dtype: Optional[str] = None):
    """``seconds`` collects each layer's host wall time (as logged)."""
    seconds = [] if seconds is None else seconds
    layers = decoder_layers(model)
    lname = next(n for n, m in model.named_modules() if m is layers)
    weights = {name: s.weights for name, (s, mod) in schemes.items() if mod is awq}
    mappings = awq.mappings or awq_mod.DEFAULT_MAPPINGS
    t0 = time.time()
    inputs = _capture_layer0_inputs(model, layers, batches)
    log.info("AWQ: layer-0 inputs of %d samples captured in %.2fs", len(inputs), time.time() - t0)
    mtype = model_type(model)
    stager = None
    batched: Optional[bool] = None  # per-sample layer calls run as one batched call (checked on layer 0)
    def onload(layer):
        nonlocal stager
        if stager is None:
            from .staging import H2DStager
            stager = H2DStager(device)
        return _onload(layer, stager)

    for i, layer in enumerate(layers):
        home = next(layer.parameters()).device
        host = None
        if residency is not None:  # rank 0 onloads if needed, then one broadcast to every rank
            host = residency.fetch(layer, onload)
        elif home != device:  # layer-by-layer onload: pinned staging, the host tensors kept for the offload
            host = onload(layer)
        t0 = time.time()
        if batched is None:
            batched = BATCH_LAYER_CALLS and _batched_forward_ok(layer, inputs)
        rep = awq_mod.awq_layer(layer, checkpoint_name(f"{lname}.{i}", mtype), inputs, mappings, weights,
                                awq.duo_scaling, awq.n_grid, mtype=mtype, calibrate_all_experts=calibrate_all_experts,
                                stateful_observers=stateful_observers, batched_calls=batched, awq_dtype=awq_dtype)
        report[f"{lname}.{i}"] = rep
        stacked = awq_mod.stack_layer_calls(inputs) if batched else None
        with awq_mod.phase("propagation"):
            if stacked is not None:  # propagate all samples in one call, split back per sample
                out = _layer_out(layer(*stacked[0], **stacked[1]))
                nxt = [((out[j:j + 1],) + tuple(args[1:]), kwargs) for j, (args, kwargs) in enumerate(inputs)]
            else:  # per sample (on QZ_CALIB_THREADS host threads / streams when set; same bits)
                outs = awq_mod.run_samples(lambda j: _layer_out(layer(*inputs[j][0], **inputs[j][1])), len(inputs))
                nxt = [((out,) + tuple(args[1:]), kwargs) for out, (args, kwargs) in zip(outs, inputs)]
        inputs = nxt
        if residency is not None:  # the other ranks keep only the tensors of their own shards
            residency.release(layer)
        if host is not None:
            _offload(layer, host)
        dt = time.time() - t0
        seconds.append(dt)
        log.info("AWQ layer %d: %d mappings in %.2fs", i, len(rep), dt)
        if awq_mod.PHASE_TIMING:
            log.info("AWQ phases so far (s): %s", {k: round(v, 3) for k, v in awq_mod.PHASES.items()})


def oneshot(model: nn.Module, recipe: Union[str, dict, list], dataset=None, processor=None,
            max_seq_length: Optional[int] = 2048, num_calibration_samples: Optional[int] = 512,
            moe_calibrate_all_experts: bool = True, device: Union[str, torch.device, None] = None,
            output_dir: Optional[str] = None, stateful_observers: bool = False,
            device_resident: Optional[bool] = None, max_shard_bytes: Optional[int] = None,
            awq_dtype: Optional[str] = None, **kwargs) -> nn.Module:
    """Apply the recipe to ``model`` in place (llmcompressor.oneshot signature as used at
    scripts/do_oneshot.py:179-187).  ``processor`` is accepted for API parity (unused: the
    dataset is already tokenized).  ``moe_calibrate_all_experts``: AWQ statistics and loss
    inputs of expert linears use every calibration token (True, the reference's setting) or
    only the tokens the router sends to that expert (False); the MoE block's own output is
    always the routed one (awq.py).  ``stateful_observers``: AWQ grid observations of balance
    layers whose scheme names ``minmax`` / ``static_minmax`` keep the observer's memory across
    the grid points (stateful reading); default memoryless (D7).
    ``device_resident``: a host-resident model is moved to ``device`` for the AWQ pass and left
    there (True), or only its decoder layers are onloaded one at a time and returned to the host
    (False, the reference's placement); default: resident when its parameters take at most
    half of the device's free memory.
    ``awq_dtype``: "bf16" (default, SURVEY A.6's reading of llmcompressor: statistics and grid
    scales in the activation dtype) or "fp32" (rounds 1-4) -- decision D8, awq.AWQ_DTYPE.

    Under torch.distributed with a meta-device skeleton on every rank but 0
    (``residency.Residency``, BASELINE configs[4]): rank 0's layers are broadcast as the pass
    reaches them and each rank keeps only the tensors of the checkpoint shards it will write
    (``max_shard_bytes``: the shard size ``save_compressed`` will be called with)."""
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device())
    device = torch.device(device)
    modifiers = parse_recipe(recipe)
    schemes = resolve_schemes(model, modifiers)
    if not schemes:
        raise ValueError("recipe targets no module of this model")
    wrong = sorted({str(ref.weight.dtype) for ref in iter_linears(model)
                    if ref.name in schemes and ref.weight.dtype != torch.bfloat16})
    if wrong:  # every kernel reads bf16: fail before any work, not inside the AWQ pass or the save
        raise ValueError(f"the MI355X kernels quantize bfloat16 weights (the reference loads its models in "
                         f"bfloat16, scripts/do_oneshot.py:88); the recipe targets {', '.join(wrong)} weights: "
                         f"load the model with torch_dtype=torch.bfloat16")
    report: Dict[str, Any] = {}
    layer_seconds: List[float] = []
    model.quantization_scheme_map = {n: s for n, (s, _) in schemes.items()}  # the residency plan reads it
    from . import residency as residency_mod
    res = None
    if residency_mod.skeleton_mode(model):
        from .compressor import SHARD_BYTES
        res = residency_mod.Residency(model, device, max_shard_bytes or SHARD_BYTES)
        model.quantization_residency = res
    awqs = [m for m in modifiers if isinstance(m, AWQModifier)]
    if awqs:
        batches = _batches(dataset, num_calibration_samples, max_seq_length, device)
        if not batches:
            raise ValueError("AWQModifier needs a calibration dataset")
        warm = _start_warmup(model, device, max(b["input_ids"].shape[1] for b in batches))
        if next(model.parameters()).device.type == "cpu" and (res is None or res.rank == 0):
            if device_resident if device_resident is not None else _fits_on_device(model, device):
                # 288 GB of HBM: a model that fits moves to the device once and stays there (no
                # per-layer onload / offload over PCIe; save_compressed then needs no staging)
                t0 = time.time()
                _to_device_staged(model, device)
                if awq_mod.PHASE_TIMING:
                    t1 = time.time()
                    torch.cuda.synchronize(device)
                    t2 = time.time()
                    torch.cuda.synchronize(device)
                    log.info("model move: enqueue %.3fs, device sync %.3fs, second sync %.3fs", t1 - t0, t2 - t1,
                             time.time() - t2)
                log.info("model moved to %s in %.2fs (%.2f GB)", device, time.time() - t0,
                         sum(p.numel() * p.element_size() for p in model.parameters()) / 1e9)
            else:
                # embeddings / rotary / final norm run on the device; layers are onloaded one
                # by one (the reference's sequential-pipeline placement)
                _to_device_except(model, decoder_layers(model), device)
        if res is not None:
            res.materialise_outside(model, decoder_layers(model))
        if warm is not None:
            warm.join()
        # MoE experts in the reference's (transformers 4.57) eager arithmetic, at grouped speed (D15)
        with bmm_guard(), eager_experts(model), fused_mlps(model) as n_mlp, fused_rmsnorms(model) as n_norm, \
                fused_rotary(model) as n_rot:
            _log_swaps(model, {"SiLU·up (dense_mlp)": n_mlp, "128-wide RMSNorm (dense_norm)": n_norm,
                               "rotary embedding (rotary)": n_rot})
            for m in awqs:
                _sequential_awq(model, m, schemes, batches, device, report, moe_calibrate_all_experts,
                                stateful_observers, residency=res, seconds=layer_seconds, awq_dtype=awq_dtype)
    elif res is not None:  # RTN: no calibration pass, but each rank still needs its shards' tensors
        stager = []

        def onload(layer):
            if not stager:
                from .staging import H2DStager
                stager.append(H2DStager(device))
            return _onload(layer, stager[0])
        res.materialise_outside(model, decoder_layers(model))
        res.distribute(model, decoder_layers(model), onload, _offload)
    if res is not None:  # helper ranks keep only the non-layer tensors they will write
        res.release_outside(model, decoder_layers(model))
    model.quantization_scheme_map = {n: s for n, (s, _) in schemes.items()}
    model.quantization_modifiers = modifiers
    model.quantization_recipe = recipe  # written next to the checkpoint as recipe.yaml
    model.awq_report = report
    model.awq_layer_seconds = layer_seconds  # per decoder layer (and AWQ modifier), as logged
    if output_dir is not None:
        from .compressor import save_compressed
        save_compressed(model, output_dir)
    return model


# model types whose transformers forwards the dense swaps restate (D16): for these a swap that
# does not engage means transformers' code changed -- the AWQ pass stays exact, only slower
_SWAP_MODEL_TYPES = ("qwen3",)


def _log_swaps(model: nn.Module, counts: Dict[str, int]) -> None:
    """One line per D16 forward swap: how many modules / functions it engaged; a warning for each
    swap that engaged nothing on a model type it was written for (patching.same_code found no
    bytecode-equal forward, e.g. after a transformers upgrade)."""
    mtype = getattr(getattr(model, "config", None), "model_type", None)
    for name, n in counts.items():
        if n:
            log.info("AWQ pass: %s swap engaged on %d module(s)", name, n)
        elif mtype in _SWAP_MODEL_TYPES:
            log.warning("AWQ pass: %s swap did NOT engage on this %s model (no forward is bytecode-equal to the "
                        "transformers code it restates); the model's own forward runs -- exact, slower", name, mtype)
        else:
            log.info("AWQ pass: %s swap not applicable to model type %s", name, mtype)


WARMUP = True  # first-call library set-up on a thread beside the model move


def _start_warmup(model: nn.Module, device, seq_len: int) -> Optional[threading.Thread]:
    """First-call costs of the capture forward, paid on a helper thread while the model moves to
    the device: the rotary embedding's f32 batched matmul ([1, head_dim / 2, 1] @ [1, 1, T]:
    0.18 s on its first call, the BLAS library's set-up), its cat / cos / sin (0.02 s) and a bf16
    linear (0.04 s) (`scripts/first_call_probe.py`), and D8's bf16 grid ops.  Nothing it computes is used."""
    if not WARMUP or torch.device(device).type != "cuda":
        return None
    cfg = getattr(model, "config", None)
    heads = getattr(cfg, "num_attention_heads", None)
    hd = getattr(cfg, "head_dim", None) or (getattr(cfg, "hidden_size", 0) // heads if heads else 128)

    @torch.no_grad()
    def run():
        a = torch.ones(1, max(hd // 2, 1), 1, device=device)
        f = (a @ torch.ones(1, 1, seq_len, device=device)).transpose(1, 2)
        e = torch.cat((f, f), dim=-1)
        e.cos(), e.sin()
        x = torch.ones(16, 256, device=device, dtype=torch.bfloat16)
        torch.nn.functional.linear(x, x)
        # D8's bf16 grid formula (pow / clamp / amax / amin / sqrt on bf16; 0.16 s of first calls
        # on layer 0 otherwise, profiles/r05s_phases_bf16.log) and running mean
        from . import awq as awq_mod
        xm = torch.ones(2, 256, device=device, dtype=torch.float32)
        for r in (0.0, 0.05, 0.5):
            awq_mod._grid_scales_bf16(xm, xm, r, True)
            awq_mod._grid_scales_bf16(xm[0], xm[0], r, False)
        awq_mod._running_mean_bf16([(xm[0], 3), (xm[1], 5)])
        torch.cuda.synchronize(device)

    th = threading.Thread(target=run, name="qz-warmup", daemon=True)
    th.start()
    return th


BATCH_LAYER_CALLS = os.environ.get("QZ_BATCH_LAYER_CALLS", "1") == "1"
HOST_COPY = "keep"  # host image of a moved model: kept with the model / "release"d (r03ae A/B)


@torch.no_grad()
def _batched_forward_ok(layer: nn.Module, inputs) -> bool:
    """Is the decoder layer's forward over the stacked samples bit-identical to its per-sample
    forwards?  (Row- and sequence-independent kernels make it so on this stack; checked once, on
    the first layer, before anything is batched.)"""
    t0 = time.time()
    stacked = awq_mod.stack_layer_calls(inputs)
    if stacked is None:
        return False
    out = _layer_out(layer(*stacked[0], **stacked[1]))

    def same(j: int) -> bool:
        p = _layer_out(layer(*inputs[j][0], **inputs[j][1]))
        if p.dtype == torch.bfloat16:
            return torch.equal(out[j:j + 1].view(torch.int16), p.view(torch.int16))
        return torch.equal(out[j:j + 1], p)
    # sample 0 first: a layer whose batched forward differs (the MoE layers' per-expert GEMMs see
    # other row counts batched) is told apart after one per-sample call instead of all of them
    ok = same(0) and all(same(j) for j in range(1, len(inputs)))
    log.info("AWQ: per-sample layer calls %s as one batched call of %d (checked in %.2fs)",
             "run" if ok else "NOT run (bits differ)", len(inputs), time.time() - t0)
    return ok


@torch.no_grad()
def _to_device_staged(model: nn.Module, device) -> None:
    """Host -> device move of every parameter / buffer through pinned staging buffers
    (``staging.H2DStager``) instead of one pageable copy per tensor: the Qwen3-4B random-init
    model's 8 GB took 7.8 s as ``model.to(device)``."""
    from .staging import H2DStager
    st = H2DStager(device)
    old: List[torch.Tensor] = []  # host storage released only after the last DMA (see below)
    for m in model.modules():
        for store in (m._parameters, m._buffers):
            for name, t in list(store.items()):
                if t is None or t.device.type != "cpu":
                    continue
                dst = st.copy(t)
                old.append(t.data if isinstance(t, nn.Parameter) else t)
                if isinstance(t, nn.Parameter):
                    t.data = dst
                else:
                    store[name] = dst
    t0 = time.time()
    st.synchronize()
    if awq_mod.PHASE_TIMING:
        log.info("model move: stager %s, stream sync %.3fs", {k: round(v, 3) for k, v in st.stats.items()},
                 time.time() - t0)
    # Unmapping host pages while DMAs run slows the DMAs ~6x on this platform (the Qwen3-4B move:
    # copy phase 1.6-1.8 s freeing as it goes vs 0.27-0.29 s deferred, profiles/r02ad_stage_probe.log),
    # and unmapping 8 GB takes ~0.6 s during which the process's memory-map lock stalls the main
    # thread's own GPU calls: released on a helper thread right after the move, the next
    # synchronise waited 0.69 s on an idle device and the layer-0 capture took 0.95 s instead of
    # 0.28 s (QZ_AWQ_PHASE_TIMING=1, scripts/gpu_r03ad.sh).  So the host image is kept with the
    # model (the reference's model lives on the host throughout anyway) and goes when the model
    # does; HOST_COPY = "release" frees it on a helper thread instead, one tensor at a time.
    if HOST_COPY == "release":
        def release():
            while old:
                old.pop()
                time.sleep(0)
        threading.Thread(target=release, name="qz-host-release", daemon=True).start()
    else:
        model._qz_host_image = old


def _onload(module: nn.Module, stager) -> Dict[tuple, torch.Tensor]:
    """Move ``module``'s host parameters / buffers to the stager's device; returns the host
    tensors (by module, kind and name of their slot) so ``_offload`` can copy the results back into them."""
    host: Dict[tuple, torch.Tensor] = {}
    for m in module.modules():
        for store in (m._parameters, m._buffers):
            for name, t in list(store.items()):
                if t is None or t.device.type != "cpu":
                    continue
                dst = stager.copy(t)
                host[(id(m), store is m._buffers, name)] = t.data if isinstance(t, nn.Parameter) else t
                if isinstance(t, nn.Parameter):
                    t.data = dst
                else:
                    store[name] = dst
    stager.wait()
    return host


def _offload(module: nn.Module, host: Dict) -> None:
    """Copy the (smoothed) device tensors back into their original host tensors and point the
    module at those again: the host pages are already resident, no new allocation."""
    for m in module.modules():
        for is_buf, store in ((False, m._parameters), (True, m._buffers)):
            for name, t in list(store.items()):
                h = host.get((id(m), is_buf, name))
                if h is None:
                    continue
                h.copy_(t.detach())
                if isinstance(t, nn.Parameter):
                    t.data = h
                else:
                    store[name] = h


def _fits_on_device(model: nn.Module, device) -> bool:
    nbytes = sum(p.numel() * p.element_size() for p in model.parameters())
    free, _ = torch.cuda.mem_get_info(torch.device(device))
    return nbytes <= free // 2


def _to_device_except(model: nn.Module, layers: nn.ModuleList, device):
    """Move everything but the decoder layers to ``device`` (layers are onloaded one at a time)."""
    inside = {id(m) for m in layers.modules()}
    for m in model.modules():
        if id(m) in inside:
            continue
        for p in m.parameters(recurse=False):
            p.data = p.data.to(device)
        for k, b in list(m.named_buffers(recurse=False)):
            setattr(m, k, b.to(device))
