"""Host-side short-batch plumbing of the S > 128 attention (CPU): the loader's token counts carry
the batch's longest sequence, graph keys separate short batches, and a captured graph sees the
same short flag as the batches that replay it (csrc/kernels/attention.hip split_mode)."""
import pickle

import torch

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (
    CICIDS2017Dataset, DeviceLoader, PackedTokens, short_batch)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine.graph import (
    GraphedTrainStep, key_tokens)


def test_packed_tokens_is_an_int_with_max_len():
    t = PackedTokens(torch.tensor(300), torch.tensor(90))
    assert t == 300 and isinstance(t, int) and t.max_len == 90
    assert (t + 64) // 64 * 64 == 320  # arithmetic gives plain ints
    u = pickle.loads(pickle.dumps(t))
    assert u == 300 and u.max_len == 90


def test_short_batch_rule():
    assert short_batch(PackedTokens(300, 128), 256)
    assert not short_batch(PackedTokens(300, 129), 256)  # one long sequence: the length split decides
    assert not short_batch(PackedTokens(300, 90), 128)   # S <= 128 runs the S <= 128 kernels anyway
    assert not short_batch(300, 256)                     # a bare count says nothing about lengths
    assert not short_batch(None, 256)


def _dataset(lens, S):
    n = len(lens)
    ids = torch.randint(1000, 2000, (n, S))
    for i, L in enumerate(lens):
        ids[i, L:] = 0
    ds = CICIDS2017Dataset.__new__(CICIDS2017Dataset)
    ds.input_ids = ids
    ds.attention_mask = (torch.arange(S)[None] < torch.tensor(lens)[:, None]).to(torch.int64)
    ds.labels = torch.zeros(n, dtype=torch.int64)
    return ds


def test_loader_token_counts_carry_the_longest_sequence():
    lens = [80, 77, 120, 5, 200, 64, 90, 33]
    for shuffle in (False, True):
        dl = DeviceLoader(_dataset(lens, 256), batch_size=4, shuffle=shuffle, seed=3)
        for b in dl:
            mask = b["attention_mask"]
            assert b["n_tokens"] == int(mask.sum())
            assert b["n_tokens"].max_len == int(mask.sum(1).max())


def test_graph_keys_separate_short_batches_and_capture_with_the_same_flag():
    st = GraphedTrainStep(lambda *a: None, warmup=1, enabled=False, bucket=lambda t, B, S: (int(t) + 63) // 64 * 64)
    ids = torch.zeros(4, 256, dtype=torch.int64)
    k_short = st._key(ids, PackedTokens(300, 100))
    k_long = st._key(ids, PackedTokens(300, 200))
    assert k_short != k_long and k_short[1] == k_long[1] == 320
    assert short_batch(key_tokens(k_short), 256) and not short_batch(key_tokens(k_long), 256)
    assert key_tokens(k_short) == 320 and key_tokens(st._key(ids, None)) is None
