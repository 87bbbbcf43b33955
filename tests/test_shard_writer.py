"""save_compressed's write plan (CPU): the checkpoint layout is fixed before anything is
compressed -- ``_unit_layout`` gives every module's on-disk tensor names and sizes (checked here
against the oracle's compress_weight for every scheme), ``save_plan`` splits them into shards and
gives each shard to one rank; ``_PlannedShardWriter`` writes a rank's shards as their tensors
arrive.  Whatever the number of ranks, the union of the files is byte-identical to one process."""
import filecmp
import json
import os

import pytest
import torch
from safetensors.torch import load_file
from torch import nn

import ct_torch as ct  # checker only
from quantizers_amd.compressor import CompressUnit, SavePlan, _PlannedShardWriter, _split_shards, _unit_layout, \
    save_plan
from quantizers_amd.model import LinearRef
from quantizers_amd.quantization import QuantizationArgs, QuantizationScheme

SCHEMES = [
    (dict(num_bits=4, type="int", symmetric=True, group_size=128), dict(group_size=128)),
    (dict(num_bits=4, type="int", symmetric=False, group_size=32), dict(symmetric=False, group_size=32)),
    (dict(num_bits=8, type="int", symmetric=False, strategy="channel"),
     dict(num_bits=8, symmetric=False, strategy="channel", group_size=None)),
    (dict(num_bits=8, type="float", group_size=32), dict(num_bits=8, type="float", group_size=32)),
    (dict(num_bits=8, type="float", strategy="block", block_structure=[128, 128]),
     dict(num_bits=8, type="float", strategy="block", block_structure=(128, 128), group_size=None)),
    (dict(num_bits=4, type="float", group_size=32, scale_dtype="uint8"),
     dict(num_bits=4, type="float", group_size=32, scale_dtype="e8m0")),
    (dict(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="float8_e4m3fn"),
     dict(num_bits=4, type="float", strategy="tensor_group", group_size=16, scale_dtype="fp8")),
]


@pytest.mark.parametrize("ours,oracle", SCHEMES)
def test_unit_layout_matches_compressed_tensors(ours, oracle):
    a = QuantizationArgs(**ours)
    sch = QuantizationScheme(targets=["Linear"], weights=a)
    g = torch.Generator().manual_seed(0)
    lin = nn.Linear(256, 256, bias=False).to(torch.bfloat16)
    lin.weight.data = (torch.randn(256, 256, generator=g) * 0.02).to(torch.bfloat16)
    dense = CompressUnit([LinearRef("m.q_proj", lin, "weight")], sch, stacked=False)
    ref = ct.compress_weight(lin.weight.data, ct.QArgs(**oracle))
    want = sorted((f"m.q_proj.{k}", v.numel() * v.element_size()) for k, v in ref.items())
    assert sorted(_unit_layout(dense)) == want
    # a stacked unit: experts' gate halves of a fused [E, 2I, H] parameter
    mod = nn.Module()
    mod.gate_up_proj = nn.Parameter((torch.randn(3, 512, 256, generator=g) * 0.02).to(torch.bfloat16))
    refs = [LinearRef(f"e.{e}.gate_proj", mod, "gate_up_proj", index=(e, slice(0, 256))) for e in range(3)]
    lay = sorted(_unit_layout(CompressUnit(refs, sch, stacked=True)))
    want = sorted((f"e.{e}.gate_proj.{k}", nb) for e in range(3) for k, nb in
                  ((k, v.numel() * v.element_size()) for k, v in ref.items()))
    assert lay == want


def _items():
    g = torch.Generator().manual_seed(0)
    return [(f"m.{i}.weight_packed", torch.randint(-100, 100, (16, 8 + i), dtype=torch.int32, generator=g))
            for i in range(10)] + [("m.big", torch.randn(64, 64, generator=g).to(torch.bfloat16))]


def _plan(items, world, max_bytes):
    order = [(n, t.numel() * t.element_size()) for n, t in items]
    shards = _split_shards(order, max_bytes)
    n = len(shards)
    files = ["model.safetensors"] if n == 1 else [f"model-{i + 1:05d}-of-{n:05d}.safetensors" for i in range(n)]
    total = sum(nb for _, nb in order)
    owner, before = [], 0
    size = dict(order)
    for names in shards:
        nb = sum(size[x] for x in names)
        owner.append(min(world - 1, int(world * (before + nb / 2) / total)))
        before += nb
    return SavePlan(order, shards, files, owner, [[] for _ in range(world)], [[] for _ in range(world)])


def test_split_closes_shards_at_the_limit():
    sh = _split_shards([("a", 500), ("b", 500), ("c", 300), ("d", 2000), ("e", 10)], 1200)
    assert sh == [["a", "b"], ["c"], ["d"], ["e"]]
    assert _split_shards([], 100) == [[]]


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_ranks_write_their_shards_union_equals_one_process(tmp_path, world):
    items = _items()
    one = tmp_path / "one"
    w = _PlannedShardWriter(str(one), _plan(items, 1, 1200), 0)
    w.add(dict(items[:4]))
    w.add(dict(items[4:]))
    n, total = w.close()
    assert n == len(items) and total == sum(t.numel() * t.element_size() for _, t in items)
    plan = _plan(items, world, 1200)
    assert len(plan.files) > 2
    multi = tmp_path / "multi"
    written = []
    for r in range(world):
        wr = _PlannedShardWriter(str(multi), plan, r)
        # every rank sees some tensors of other ranks' shards (straddling units): dropped
        wr.add(dict(items[::2]))
        wr.add(dict(items[1::2]))
        wr.close()
        written.append({s for s, o in enumerate(plan.owner) if o == r})
    files = sorted(os.listdir(multi))
    assert files == sorted(plan.files) and not any(f.endswith(".tmp") for f in os.listdir(multi))
    assert sorted(os.listdir(one)) == files
    for f in files:
        assert filecmp.cmp(one / f, multi / f, shallow=False), f
    if world > 1:
        assert sum(1 for s in written if s) > 1  # more than one rank wrote
    got = {}
    for f in files:
        part = load_file(str(multi / f))
        assert sum(t.numel() * t.element_size() for t in part.values()) <= 1200 or len(part) == 1
        got.update(part)
    for name, t in items:
        assert torch.equal(got[name], t)


def test_missing_or_resized_tensor_is_an_error(tmp_path):
    items = _items()
    plan = _plan(items, 1, 1 << 30)
    w = _PlannedShardWriter(str(tmp_path / "a"), plan, 0)
    w.add(dict(items[:-1]))
    with pytest.raises(RuntimeError, match="never completed"):
        w.close()
    w = _PlannedShardWriter(str(tmp_path / "b"), plan, 0)
    with pytest.raises(ValueError, match="the plan expected"):
        w.add({items[0][0]: torch.zeros(3, dtype=torch.int32)})
    w.pool.shutdown()


def _tiny_model():
    torch.manual_seed(0)
    m = nn.Module()
    m.model = nn.Module()
    m.model.layers = nn.ModuleList()
    for _ in range(4):
        blk = nn.Module()
        blk.q_proj = nn.Linear(64, 96, bias=False)
        blk.up_proj = nn.Linear(64, 128, bias=True)
        blk.norm = nn.LayerNorm(64)
        m.model.layers.append(blk)
    m.to(torch.bfloat16)
    sch = QuantizationScheme(targets=["Linear"], weights=QuantizationArgs(num_bits=4, type="int", symmetric=True,
                                                                          group_size=32))
    m.quantization_scheme_map = {f"model.layers.{i}.{p}": sch for i in range(4) for p in ("q_proj", "up_proj")}
    return m


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_save_plan_assigns_units_and_raw_to_shard_owners(world):
    from quantizers_amd.compressor import compression_units
    units, raw = compression_units(_tiny_model())
    plan = save_plan(units, raw, world, max_shard_bytes=3000)
    names = [n for n, _ in plan.order]
    assert len(names) == len(set(names)) and sum(plan.shards, []) == names
    assert plan.owner == sorted(plan.owner) and all(0 <= r < world for r in plan.owner)
    wmap = plan.weight_map()
    for r in range(world):
        mine = {n for s, o in enumerate(plan.owner) if o == r for n in plan.shards[s]}
        covered = {n for i in plan.units_of[r] for n, _ in _unit_layout(units[i])} | set(plan.raw_of[r])
        assert mine <= covered  # everything a rank writes, it produces
        for i in plan.units_of[r]:  # and it compresses nothing that has no tensor in its shards
            assert {n for n, _ in _unit_layout(units[i])} & mine
    assert set(wmap) == set(names) and set(raw) <= set(names)
    # bytes per rank are balanced to within one shard
    per = [sum(nb for s, o in enumerate(plan.owner) if o == r for nb in
               (dict(plan.order)[n] for n in plan.shards[s])) for r in range(world)]
    biggest = max(sum(dict(plan.order)[n] for n in sh) for sh in plan.shards)
    if len(plan.shards) >= world:
        assert max(per) - min(per) <= 2 * biggest
