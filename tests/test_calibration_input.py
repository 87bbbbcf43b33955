"""oneshot's calibration input (CPU): the tokenized `datasets.Dataset` the reference's
calibration-set loader produces (columns input_ids / attention_mask, do_oneshot.py:174-187)
is accepted as is, as are lists of dicts and [N, S] tensors; truncation and sample limits
follow max_seq_length / num_calibration_samples."""
import torch

from quantizers_amd.oneshot import _batches


def test_hf_dataset_rows():
    from datasets import Dataset
    ds = Dataset.from_dict({"input_ids": [[1, 2, 3, 4, 5], [6, 7, 8]],
                            "attention_mask": [[1, 1, 1, 1, 1], [1, 1, 0]]})
    b = _batches(ds, num_samples=None, max_seq_length=4, device="cpu")
    assert len(b) == 2
    assert b[0]["input_ids"].tolist() == [[1, 2, 3, 4]] and b[0]["attention_mask"].tolist() == [[1, 1, 1, 1]]
    assert b[1]["input_ids"].tolist() == [[6, 7, 8]] and b[1]["attention_mask"].tolist() == [[1, 1, 0]]


def test_sample_limit_and_tensor_input():
    t = torch.arange(30).reshape(5, 6)
    b = _batches(t, num_samples=3, max_seq_length=None, device="cpu")
    assert len(b) == 3 and b[2]["input_ids"].tolist() == [[12, 13, 14, 15, 16, 17]]
    assert _batches(None, 4, 8, "cpu") == []
    rows = [{"input_ids": [9, 9]}, {"input_ids": torch.tensor([1, 2, 3])}]
    b = _batches(rows, None, 2, "cpu")
    assert [x["input_ids"].tolist() for x in b] == [[[9, 9]], [[1, 2]]]
