"""Data layer: synthetic CICIDS2017 shape, featuriser template, preprocessing, splits."""
import math

import numpy as np
import pandas as pd
import pytest

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (
    CICIDS2017_COLUMNS, features_to_text, generate_cicids2017, preprocess_data, render_texts, split_60_20_20,
    write_csv)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import _text_native
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data.synthetic import (
    dedup_columns)

REF_HEADER = open("/root/reference/CICIDS2017.csv").readline().rstrip("\n").split(",") \
    if __import__("os").path.exists("/root/reference/CICIDS2017.csv") else None


def test_header_matches_reference_csv():
    assert len(CICIDS2017_COLUMNS) == 79
    if REF_HEADER is not None:
        assert CICIDS2017_COLUMNS == REF_HEADER
    assert " Flow IAT Max" in CICIDS2017_COLUMNS and CICIDS2017_COLUMNS.count("Fwd Header Length") == 2


def test_synthetic_shape_and_balance(tmp_path):
    df = generate_cicids2017(20000, seed=1)
    assert list(df.columns) == dedup_columns(CICIDS2017_COLUMNS)
    frac = (df["Label"] == "DDoS").mean()
    assert 0.54 < frac < 0.60
    assert np.isinf(df["Flow Bytes/s"].to_numpy()).any() or df["Flow Bytes/s"].isna().any()
    assert (df.loc[df.Label == "DDoS", "Destination Port"] == 80).all()
    p = tmp_path / "c.csv"
    write_csv(df.head(50), str(p))
    back = pd.read_csv(p)
    assert list(back.columns) == dedup_columns(CICIDS2017_COLUMNS)
    assert np.allclose(back["Flow Duration"].to_numpy(), df.head(50)["Flow Duration"].to_numpy())


def test_generator_is_deterministic():
    a = generate_cicids2017(1000, seed=7)
    b = generate_cicids2017(1000, seed=7)
    pd.testing.assert_frame_equal(a, b)


def _row():
    return pd.Series({"Destination Port": 54865, "Flow Duration": 3, "Total Fwd Packets": 2,
                      "Total Backward Packets": 0, "Total Length of Fwd Packets": 12,
                      "Total Length of Bwd Packets": 0, "Fwd Packet Length Max": 6, "Fwd Packet Length Min": 6,
                      "Flow Bytes/s": 4000000.0, "Flow Packets/s": 666666.6667}, dtype=object)


def test_features_to_text_template():
    # client1.py:69-80 verbatim; first data row of the committed CSV.
    expect = ("Destination port is 54865. Flow duration is 3 microseconds. Total forward packets are 2. "
              "Total backward packets are 0. Total length of forward packets is 12 bytes. "
              "Total length of backward packets is 0 bytes. Maximum forward packet length is 6. "
              "Minimum forward packet length is 6. Flow bytes per second is 4000000.0. "
              "Flow packets per second is 666666.6667.")
    assert features_to_text(_row()) == expect


def test_render_texts_matches_rowwise_apply():
    df = generate_cicids2017(400, seed=3)
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data.featurize import (
        clean_frame)
    df = clean_frame(df)
    ref = df.apply(features_to_text, axis=1).tolist()
    assert render_texts(df, native=False) == ref
    if _text_native.load() is not None:
        assert render_texts(df, native=True) == ref


@pytest.mark.skipif(_text_native.load() is None, reason="native text ext not built")
def test_native_float_repr_matches_python():
    ext = _text_native.load()
    rng = np.random.default_rng(0)
    vals = [0.0, -0.0, 1.0, 0.1, 1e16, 1e15, 123456789012345.6, 1.5e-5, 0.0001, 0.00012, 1e-300, 5e-324,
            1.7976931348623157e308, 4000000.0, 666666.6667, float("inf"), float("-inf"), 2.5, -3.75, 1e22]
    vals += list(rng.standard_normal(200) * 10.0 ** rng.integers(-8, 18, 200))
    for v in vals:
        assert ext.py_repr(float(v)) == repr(float(v)), v
    assert ext.py_repr(float("nan")) == "nan"


def test_preprocess_handles_inf_and_samples():
    df = generate_cicids2017(5000, seed=2)
    df.loc[df.index[:5], "Flow Bytes/s"] = np.inf
    texts, labels = preprocess_data(df, data_fraction=0.1, seed=42)
    assert len(texts) == 500 and len(labels) == 500
    assert not any("inf" in t for t in texts)
    assert set(labels) <= {0, 1}


def test_split_sizes_match_reference():
    # 22,574 sampled rows -> 13,544 / 4,515 / 4,515 (client1_terminal_output.txt)
    n = 22574
    (a, _), (b, _), (c, _) = split_60_20_20(list(range(n)), [0] * n, 42)
    assert (len(a), len(b), len(c)) == (13544, 4515, 4515)


REF_CSV = "/root/reference/CICIDS2017.csv"


@pytest.mark.skipif(not __import__("os").path.exists(REF_CSV), reason="reference CSV not mounted")
@pytest.mark.parametrize("seed", [42, 43])
def test_preprocess_reference_csv_parity(seed):
    """The reference's own committed sample (2,885 rows, 3 with Infinity) through our
    preprocess_data == the reference pipeline written out in plain pandas (client1.py:68-93):
    inf -> NaN -> column mean, 10 % sample with the client seed, the 10-sentence template."""
    texts, labels = preprocess_data(REF_CSV, data_fraction=0.1, seed=seed)
    df = pd.read_csv(REF_CSV)
    df = df.replace([np.inf, -np.inf], np.nan)
    df = df.fillna(df.mean(numeric_only=True))
    df = df.sample(frac=0.1, random_state=seed)

    def row_text(r):
        return (f"Destination port is {r['Destination Port']}. Flow duration is {r['Flow Duration']} microseconds. "
                f"Total forward packets are {r['Total Fwd Packets']}. "
                f"Total backward packets are {r['Total Backward Packets']}. "
                f"Total length of forward packets is {r['Total Length of Fwd Packets']} bytes. "
                f"Total length of backward packets is {r['Total Length of Bwd Packets']} bytes. "
                f"Maximum forward packet length is {r['Fwd Packet Length Max']}. "
                f"Minimum forward packet length is {r['Fwd Packet Length Min']}. "
                f"Flow bytes per second is {r['Flow Bytes/s']}. Flow packets per second is {r['Flow Packets/s']}.")
    ref_texts = df.apply(row_text, axis=1).tolist()
    ref_labels = df["Label"].apply(lambda x: 1 if x == "DDoS" else 0).tolist()
    assert len(texts) == len(ref_texts) == round(0.1 * len(pd.read_csv(REF_CSV)))
    assert texts == ref_texts
    assert labels == ref_labels and set(labels) == {0}  # the committed sample is all BENIGN


def test_device_loader_blocked_batches_keep_order_and_layout():
    """Full batches come from one per-epoch buffer (ids | mask | labels back to back) with the
    same rows, order and token counts as a per-batch gather; the short tail batch does not."""
    import torch
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd import data
    from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.engine.graph import (
        contiguous_block, static_block)
    df = data.generate_cicids2017(600, seed=1)
    ds = data.build_client_data(df, 0, data_fraction=1.0, max_len=64).train
    for shuffle in (False, True):
        L = data.DeviceLoader(ds, 32, shuffle=shuffle, seed=3)
        perm = torch.randperm(L.n, generator=torch.Generator().manual_seed(3)) if shuffle else torch.arange(L.n)
        for i, b in enumerate(L):
            idx = perm[i * 32:(i + 1) * 32]
            assert torch.equal(b["input_ids"], ds.input_ids[idx])
            assert torch.equal(b["attention_mask"], ds.attention_mask[idx])
            assert torch.equal(b["labels"], ds.labels[idx])
            assert b["n_tokens"] == int(ds.attention_mask[idx].sum())
            blk = contiguous_block(b["input_ids"], b["attention_mask"], b["labels"])
            assert (blk is not None) == (len(idx) == 32)
            if blk is not None:
                (si, sm, sl), flat = static_block(b["input_ids"], b["attention_mask"], b["labels"])
                flat.zero_()
                flat.copy_(blk)  # one copy refreshes all three static inputs
                assert torch.equal(si, b["input_ids"]) and torch.equal(sm, b["attention_mask"])
                assert torch.equal(sl, b["labels"])
