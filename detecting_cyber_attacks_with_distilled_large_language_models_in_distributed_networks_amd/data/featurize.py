"""Tabular -> text featuriser and CSV preprocessing (reference L0/L1).

``features_to_text`` reproduces client1.py:68-81 exactly (the 10-sentence
template; integer columns print as ints, float columns with Python ``repr``).
``preprocess_data`` reproduces client1.py:84-93: read CSV, +-inf -> NaN,
NaN -> numeric column mean, ``df.sample(frac, random_state=seed)``, render text,
label = 1 iff Label == 'DDoS'.

The reference renders with a row-wise ``df.apply`` (~1.2 s per 22k rows,
SURVEY 3.1).  ``render_texts`` is the columnar equivalent and, when the native
text extension is built, the formatting runs in C++ (csrc/text/text_native.cpp).
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple, Union

import numpy as np
import pandas as pd

TEXT_FIELDS = [
    ("Destination port is {}. ", "Destination Port"),
    ("Flow duration is {} microseconds. ", "Flow Duration"),
    ("Total forward packets are {}. ", "Total Fwd Packets"),
    ("Total backward packets are {}. ", "Total Backward Packets"),
    ("Total length of forward packets is {} bytes. ", "Total Length of Fwd Packets"),
    ("Total length of backward packets is {} bytes. ", "Total Length of Bwd Packets"),
    ("Maximum forward packet length is {}. ", "Fwd Packet Length Max"),
    ("Minimum forward packet length is {}. ", "Fwd Packet Length Min"),
    ("Flow bytes per second is {}. ", "Flow Bytes/s"),
    ("Flow packets per second is {}.", "Flow Packets/s"),
]
FEATURE_COLUMNS = [c for _, c in TEXT_FIELDS]


def features_to_text(row) -> str:
    """Exact template of client1.py:68-81 for one row (Series or mapping)."""
    return "".join(fmt.format(row[col]) for fmt, col in TEXT_FIELDS)


def _column_strings(values: np.ndarray) -> List[str]:
    if np.issubdtype(values.dtype, np.integer):
        return [str(v) for v in values.tolist()]
    if np.issubdtype(values.dtype, np.floating):
        return [repr(v) for v in values.astype(np.float64).tolist()]
    return [str(v) for v in values.tolist()]


def render_texts(df: pd.DataFrame, native: Optional[bool] = None) -> List[str]:
    """Columnar ``df.apply(features_to_text, axis=1)`` (same strings)."""
    if native is None or native:
        try:
            from . import _text_native
            ext = _text_native.load()
        except Exception:
            if native:
                raise
            ext = None
        if ext is not None:
            cols, is_int = [], []
            for c in FEATURE_COLUMNS:
                v = df[c].to_numpy()
                if np.issubdtype(v.dtype, np.integer):
                    cols.append(np.ascontiguousarray(v.astype(np.float64)))
                    is_int.append(True)
                else:
                    cols.append(np.ascontiguousarray(v.astype(np.float64)))
                    is_int.append(False)
            return ext.render_texts(cols, is_int)
    parts = [_column_strings(df[c].to_numpy()) for c in FEATURE_COLUMNS]
    fmts = [f for f, _ in TEXT_FIELDS]
    out = []
    for i in range(len(df)):
        out.append("".join(fmts[j].format(parts[j][i]) for j in range(len(fmts))))
    return out


def clean_frame(df: pd.DataFrame) -> pd.DataFrame:
    """+-inf -> NaN -> column mean (client1.py:87-88)."""
    df = df.replace([np.inf, -np.inf], np.nan)
    return df.fillna(df.mean(numeric_only=True))


def preprocess_data(source: Union[str, pd.DataFrame], data_fraction: float = 0.1,
                    seed: int = 42, native: Optional[bool] = None,
                    log=None) -> Tuple[List[str], List[int]]:
    """client1.py:84-93.  ``source`` is a CSV path or an in-memory frame."""
    if log:
        log("Starting data preprocessing")
    df = pd.read_csv(source) if isinstance(source, str) else source
    df = clean_frame(df)
    df = df.sample(frac=data_fraction, random_state=seed)
    texts = render_texts(df, native=native)
    labels = (df["Label"].to_numpy() == "DDoS").astype(np.int64).tolist()
    if log:
        log("Finished data preprocessing")
    return texts, labels


def split_60_20_20(texts: Sequence, labels: Sequence, seed: int = 42):
    """train_test_split(test_size=0.4, rs) then halve the 40 % (client1.py:365-366)."""
    from sklearn.model_selection import train_test_split
    x_tr, x_tmp, y_tr, y_tmp = train_test_split(list(texts), list(labels), test_size=0.4,
                                                random_state=seed)
    x_va, x_te, y_va, y_te = train_test_split(x_tmp, y_tmp, test_size=0.5, random_state=seed)
    return (x_tr, y_tr), (x_va, y_va), (x_te, y_te)
