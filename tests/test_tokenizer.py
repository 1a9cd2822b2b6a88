"""WordPiece tokenizer: native C++ == Python spec == HF `tokenizers` BertWordPiece (golden)."""
import random
import string

import numpy as np
import pytest

from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data import (
    WordPieceTokenizer, generate_cicids2017, render_texts)
from detecting_cyber_attacks_with_distilled_large_language_models_in_distributed_networks_amd.data.vocab import (
    CLS_ID, PAD_ID, SEP_ID, UNK_ID, VOCAB_SIZE, build_vocab)


def _texts(n=200):
    df = generate_cicids2017(n, seed=5).replace([np.inf, -np.inf], np.nan).fillna(0)
    texts = render_texts(df)
    rnd = random.Random(0)
    for _ in range(100):
        k = rnd.randint(0, 60)
        texts.append("".join(rnd.choice(string.ascii_letters + string.digits + string.punctuation + "  \t")
                             for _ in range(k)))
    texts += ["", "   ", "Hello, World!!", "x" * 150, "DDoS ATTACK at port 80."]
    return texts


def test_vocab_layout():
    v = build_vocab()
    assert len(v) == VOCAB_SIZE
    assert v[PAD_ID] == "[PAD]" and v[UNK_ID] == "[UNK]" and v[CLS_ID] == "[CLS]" and v[SEP_ID] == "[SEP]"
    assert len(set(v)) == len(v)


def test_native_matches_python_spec():
    nat = WordPieceTokenizer(native=None)
    if not nat.is_native:
        pytest.skip("native text ext not built")
    py = WordPieceTokenizer(native=False)
    texts = _texts()
    ids_n, lens_n = nat.encode_batch(texts, 128)
    ids_p, lens_p = py.encode_batch(texts, 128)
    assert np.array_equal(ids_n, ids_p) and np.array_equal(lens_n, lens_p)
    for t in texts[:50]:
        assert nat.tokenize(t) == py.tokenize_py(t)


def test_matches_hf_tokenizers_golden():
    tokenizers = pytest.importorskip("tokenizers")
    from tokenizers import Tokenizer, models, normalizers, pre_tokenizers
    vocab = {t: i for i, t in enumerate(build_vocab())}
    hf = Tokenizer(models.WordPiece(vocab, unk_token="[UNK]", max_input_chars_per_word=100))
    hf.normalizer = normalizers.BertNormalizer(clean_text=True, handle_chinese_chars=False, strip_accents=False,
                                               lowercase=True)
    hf.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    ours = WordPieceTokenizer()
    for t in _texts(100):
        assert ours.tokenize(t) == hf.encode(t, add_special_tokens=False).tokens, t


def test_call_api_shapes():
    tok = WordPieceTokenizer()
    enc = tok("Destination port is 80. Flow duration is 5 microseconds.", max_length=128, return_tensors="pt")
    assert enc["input_ids"].shape == (1, 128) and enc["attention_mask"].shape == (1, 128)
    ids = enc["input_ids"][0].tolist()
    n = int(enc["attention_mask"].sum())
    assert ids[0] == CLS_ID and ids[n - 1] == SEP_ID and all(i == PAD_ID for i in ids[n:])


def test_truncation_keeps_sep():
    tok = WordPieceTokenizer()
    ids, lens = tok.encode_batch(["word " * 500], 64)
    assert lens[0] == 64 and ids[0, 0] == CLS_ID and ids[0, 63] == SEP_ID


def test_featurized_sequence_length():
    tok = WordPieceTokenizer()
    df = generate_cicids2017(300, seed=9).replace([np.inf, -np.inf], np.nan).fillna(0)
    _, lens = tok.encode_batch(render_texts(df), 128)
    assert 70 <= lens.mean() <= 128
