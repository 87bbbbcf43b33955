"""AWQ parent-call batching (awq._batchwise_concat): a self-attention parent's per-sample
calibration calls stacked along the batch dimension give the same per-sample outputs (fp32, CPU,
transformers' Qwen3 attention with its own masks / rotary embeddings), and calls that differ
in anything but hidden_states are left alone."""
import pytest
import torch

transformers = pytest.importorskip("transformers")


def _tiny_qwen3():
    from transformers import Qwen3Config, Qwen3ForCausalLM
    cfg = Qwen3Config(hidden_size=64, intermediate_size=128, num_hidden_layers=1, num_attention_heads=4,
                      num_key_value_heads=2, head_dim=16, vocab_size=97, max_position_embeddings=128)
    torch.manual_seed(0)
    return Qwen3ForCausalLM(cfg).float().eval()


@torch.no_grad()
def test_attention_calls_batched_equal_per_sample():
    from quantizers_amd import awq
    model = _tiny_qwen3()
    attn = model.model.layers[0].self_attn
    cache = awq._ParentCache(attn)
    g = torch.Generator().manual_seed(1)
    for _ in range(5):
        model(input_ids=torch.randint(0, 97, (1, 24), generator=g), use_cache=False)  # as oneshot does
    cache.remove()
    calls = cache.calls
    assert len(calls) == 5
    batched = awq._batchwise_concat(calls, max_tokens=2 * 24)  # chunks of 2, 2, 1 sequences
    assert [c[1]["hidden_states"].shape[0] if c[1] else c[0][0].shape[0] for c in batched] == [2, 2, 1]
    ref = torch.cat(awq._run_parent(attn, calls), dim=0)
    got = torch.cat(awq._run_parent(attn, batched), dim=0)
    torch.testing.assert_close(got, ref, rtol=1e-5, atol=1e-6)


def test_calls_with_different_kwargs_are_not_batched():
    from quantizers_amd import awq
    h = [torch.randn(1, 8, 4) for _ in range(3)]
    pe = (torch.randn(1, 8, 2), torch.randn(1, 8, 2))
    calls = [((), {"hidden_states": x, "position_embeddings": pe, "attention_mask": None}) for x in h]
    assert len(awq._batchwise_concat(calls)) == 1
    other = (torch.randn(1, 8, 2), pe[1])
    calls[1] = ((), {"hidden_states": h[1], "position_embeddings": other, "attention_mask": None})
    assert awq._batchwise_concat(calls) is calls
    ragged = [((), {"hidden_states": torch.randn(1, n, 4)}) for n in (8, 9)]
    assert awq._batchwise_concat(ragged) is ragged
