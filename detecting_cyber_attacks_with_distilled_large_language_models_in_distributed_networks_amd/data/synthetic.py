"""Seeded synthetic CICIDS2017-shaped flow generator.

The committed reference CSV (/root/reference/CICIDS2017.csv) is a 2,885-row,
all-BENIGN truncation; the published run used the full Friday-afternoon DDoS
file (~225,745 rows, ~57 % DDoS).  There is no network to fetch
it, so this module produces a file of the same *shape*:

* the exact 79-column header, including the leading-space quirks
  (' Flow IAT Max', ' SYN Flag Count', ...) and the duplicated
  'Fwd Header Length' column (CICIDS2017.csv:1);
* ~57 % 'DDoS' rows, the rest 'BENIGN';
* a few 'Infinity'/NaN cells in 'Flow Bytes/s' / 'Flow Packets/s' (zero-duration
  flows), which the reference's +-inf -> NaN -> mean step handles
  (client1.py:87-88);
* class-conditional distributions that make the label recoverable from the 10
  features the reference renders to text (port, packet counts/lengths, rates),
  with a small overlap so accuracy saturates near, not at, 100 %.

DDoS rows mimic the Friday LOIC HTTP flood (port 80, few small forward packets,
large backward payloads); BENIGN rows mix DNS (53), HTTPS (443), HTTP (80) and
ephemeral-port traffic.
"""
from __future__ import annotations

import numpy as np
import pandas as pd

# Exact header of CICIDS2017.csv:1 (79 columns, leading spaces preserved).
CICIDS2017_COLUMNS = [
    "Destination Port", "Flow Duration", "Total Fwd Packets", "Total Backward Packets",
    "Total Length of Fwd Packets", "Total Length of Bwd Packets", "Fwd Packet Length Max",
    "Fwd Packet Length Min", "Fwd Packet Length Mean", "Fwd Packet Length Std",
    "Bwd Packet Length Max", "Bwd Packet Length Min", "Bwd Packet Length Mean",
    "Bwd Packet Length Std", "Flow Bytes/s", "Flow Packets/s", "Flow IAT Mean", "Flow IAT Std",
    " Flow IAT Max", "Flow IAT Min", "Fwd IAT Total", "Fwd IAT Mean", "Fwd IAT Std", "Fwd IAT Max",
    " Fwd IAT Min", "Bwd IAT Total", "Bwd IAT Mean", "Bwd IAT Std", "Bwd IAT Max", " Bwd IAT Min",
    "Fwd PSH Flags", "Bwd PSH Flags", "Fwd URG Flags", "Bwd URG Flags", "Fwd Header Length",
    "Bwd Header Length", "Fwd Packets/s", " Bwd Packets/s", " Min Packet Length",
    " Max Packet Length", "Packet Length Mean", "Packet Length Std", "Packet Length Variance",
    "FIN Flag Count", " SYN Flag Count", "RST Flag Count", "PSH Flag Count", "ACK Flag Count",
    "URG Flag Count", "CWE Flag Count", "ECE Flag Count", "Down/Up Ratio", "Average Packet Size",
    "Avg Fwd Segment Size", "Avg Bwd Segment Size", "Fwd Header Length", "Fwd Avg Bytes/Bulk",
    "Fwd Avg Packets/Bulk", "Fwd Avg Bulk Rate", "Bwd Avg Bytes/Bulk", "Bwd Avg Packets/Bulk",
    "Bwd Avg Bulk Rate", "Subflow Fwd Packets", "Subflow Fwd Bytes", "Subflow Bwd Packets",
    "Subflow Bwd Bytes", "Init_Win_bytes_forward", "Init_Win_bytes_backward", "act_data_pkt_fwd",
    "min_seg_size_forward", "Active Mean", "Active Std", "Active Max", "Active Min", "Idle Mean",
    "Idle Std", "Idle Max", "Idle Min", "Label",
]
assert len(CICIDS2017_COLUMNS) == 79


def dedup_columns(cols):
    """pandas.read_csv's mangle of duplicate names ('X' -> 'X', 'X.1', ...)."""
    seen, out = {}, []
    for c in cols:
        if c in seen:
            seen[c] += 1
            out.append(f"{c}.{seen[c]}")
        else:
            seen[c] = 0
            out.append(c)
    return out


DDOS_FRACTION = 0.57     # 2,586 / 4,515 test positives
INF_FRACTION = 0.001     # 3 of 2,885 committed rows carry 'Infinity'


HARD_OVERLAP = 0.04      # "hard" profile: irreducible label noise (~1.7 % of rows)
HARD_LOOKALIKE = 0.30    # "hard" profile: BENIGN HTTP flows shaped like the flood
# "calibrated" profile: only a few look-alike BENIGN flows (no extra label noise), sized so a
# client's 3-epoch local model lands near the reference's local 99.05-99.09 % test accuracy
# (client{1,2}_local_metrics.csv:2), where one FedAvg round has room to lift it
CALIBRATED_LOOKALIKE = 0.06
PROFILES = {"default": {}, "calibrated": {"lookalike": CALIBRATED_LOOKALIKE}, "hard": {"hard": True}}


def generate_cicids2017(n_rows: int = 225_745, seed: int = 0,
                        ddos_fraction: float = DDOS_FRACTION,
                        overlap: float = 0.0004, hard: bool = False, lookalike: float = 0.0,
                        profile: str = "") -> pd.DataFrame:
    """Return a DataFrame with CICIDS2017 columns (pandas-deduplicated names).

    ``overlap`` is the fraction of BENIGN rows drawn from the DDoS feature
    distribution (irreducible error; ~0.04 % -> accuracy ceiling ~99.98 %).

    ``hard=True`` is a profile for numerics tests whose accuracy must land well
    below 100 % so a loss curve carries information: overlap rises to
    ``HARD_OVERLAP`` and ``HARD_LOOKALIKE`` of the remaining BENIGN rows become
    port-80 flows with the flood's packet counts and small forward packets, told
    apart only by a backward payload that is drawn from a wider range (and from
    the flood's own payload values a third of the time).  The default profile's
    rows are unchanged (the look-alikes are drawn from a separate RNG stream).

    ``lookalike`` > 0 (without ``hard``): that fraction of the BENIGN rows become the look-alike
    flows, with the default label noise.  ``profile``: a named setting of ``PROFILES`` --
    "default", "calibrated" (lookalike = CALIBRATED_LOOKALIKE) or "hard".
    """
    if profile:
        if profile not in PROFILES:
            raise ValueError(f"unknown data profile {profile!r} (one of {sorted(PROFILES)})")
        kw = PROFILES[profile]
        hard = hard or kw.get("hard", False)
        lookalike = lookalike or kw.get("lookalike", 0.0)
    if hard and overlap == 0.0004:
        overlap = HARD_OVERLAP
    rng = np.random.default_rng(seed)
    n = int(n_rows)
    is_ddos = rng.random(n) < ddos_fraction
    looks_ddos = is_ddos | (rng.random(n) < overlap)

    port = np.empty(n, np.int64)
    dur = np.empty(n, np.int64)
    nfwd = np.empty(n, np.int64)
    nbwd = np.empty(n, np.int64)
    fwd_max = np.empty(n, np.int64)
    fwd_min = np.empty(n, np.int64)
    bwd_max = np.empty(n, np.int64)
    bwd_min = np.empty(n, np.int64)
    fwd_len = np.empty(n, np.int64)
    bwd_len = np.empty(n, np.int64)

    # ---- DDoS-like rows: LOIC HTTP flood -----------------------------------------------
    d = np.flatnonzero(looks_ddos)
    nd = d.size
    port[d] = 80
    dur[d] = np.exp(rng.uniform(np.log(5e2), np.log(1.2e8), nd)).astype(np.int64)
    nfwd[d] = rng.integers(1, 9, nd)
    nbwd[d] = np.where(rng.random(nd) < 0.2, 0, rng.integers(3, 8, nd))
    fwd_max[d] = rng.choice(np.array([0, 6, 20]), nd, p=[0.3, 0.3, 0.4])
    fwd_min[d] = 0
    fwd_len[d] = np.minimum(fwd_max[d] * rng.integers(1, 3, nd), fwd_max[d] * nfwd[d])
    bwd_pay = rng.choice(np.array([11595, 11601, 11607, 5840, 7300]), nd, p=[0.3, 0.3, 0.2, 0.1, 0.1])
    bwd_len[d] = np.where(nbwd[d] > 0, bwd_pay, 0)
    bwd_max[d] = np.where(nbwd[d] > 0, np.minimum(bwd_len[d], 5840 + rng.integers(0, 2, nd) * 1460), 0)
    bwd_min[d] = 0

    # ---- BENIGN rows: DNS / HTTPS / HTTP / ephemeral --------------------------------------
    b = np.flatnonzero(~looks_ddos)
    nb = b.size
    kind = rng.choice(4, nb, p=[0.35, 0.3, 0.15, 0.2])
    pb = np.where(kind == 0, 53, np.where(kind == 1, 443, np.where(kind == 2, 80,
                  rng.integers(1024, 65536, nb))))
    port[b] = pb
    # DNS: 1-2 packets each way, short.
    nf = np.where(kind == 0, rng.integers(1, 3, nb), rng.integers(2, 40, nb))
    nbk = np.where(kind == 0, rng.integers(1, 3, nb), rng.integers(1, 40, nb))
    fmax = np.where(kind == 0, rng.integers(28, 80, nb), rng.integers(100, 1461, nb))
    fmin = np.where(kind == 0, fmax - rng.integers(0, 10, nb), rng.integers(0, 60, nb))
    fmin = np.clip(fmin, 0, fmax)
    bmax = np.where(kind == 0, rng.integers(60, 300, nb), rng.integers(0, 1461, nb))
    flen = np.maximum(fmax, (fmin + fmax) // 2 * nf)
    blen = (bmax * rng.uniform(0.2, 1.0, nb) * nbk).astype(np.int64)
    nfwd[b], nbwd[b] = nf, nbk
    fwd_max[b], fwd_min[b] = fmax, fmin
    bwd_max[b], bwd_min[b] = bmax, np.minimum(bmax, rng.integers(0, 40, nb))
    fwd_len[b], bwd_len[b] = flen, blen
    dur[b] = np.where(kind == 0, rng.integers(20, 200_000, nb),
                      np.exp(rng.uniform(np.log(3), np.log(1.2e8), nb)).astype(np.int64))

    if hard or lookalike > 0:
        _lookalikes(np.random.default_rng(seed + 1_000_003), b, port, dur, nfwd, nbwd, fwd_max, fwd_min,
                    fwd_len, bwd_len, bwd_max, bwd_min, HARD_LOOKALIKE if hard else lookalike)

    # Zero-duration flows -> Infinity rates (client1.py:87 handles them).
    zero = rng.random(n) < INF_FRACTION
    dur[zero] = 0
    with np.errstate(divide="ignore", invalid="ignore"):
        bytes_s = (fwd_len + bwd_len).astype(np.float64) / dur.astype(np.float64) * 1e6
        pkts_s = (nfwd + nbwd).astype(np.float64) / dur.astype(np.float64) * 1e6
        fwd_pkts_s = nfwd.astype(np.float64) / dur * 1e6
        bwd_pkts_s = nbwd.astype(np.float64) / dur * 1e6
    both_zero = zero & ((fwd_len + bwd_len) == 0)
    bytes_s[both_zero] = np.nan
    bytes_s = np.round(bytes_s, 4)
    pkts_s = np.round(pkts_s, 5)
    fwd_pkts_s = np.round(fwd_pkts_s, 5)
    bwd_pkts_s = np.round(bwd_pkts_s, 5)

    nf_safe = np.maximum(nfwd, 1)
    nb_safe = np.maximum(nbwd, 1)
    fwd_mean = np.round(fwd_len / nf_safe, 6)
    bwd_mean = np.where(nbwd > 0, np.round(bwd_len / nb_safe, 6), 0.0)
    fwd_std = np.round(np.abs(fwd_max - fwd_min) * rng.uniform(0, 0.6, n), 6)
    bwd_std = np.round(np.abs(bwd_max - bwd_min) * rng.uniform(0, 0.6, n), 6)
    npk = nfwd + nbwd
    iat_mean = np.round(dur / np.maximum(npk - 1, 1), 6)
    iat_std = np.round(iat_mean * rng.uniform(0, 1.5, n), 6)
    iat_max = np.minimum(dur, (iat_mean * rng.uniform(1, 3, n)).astype(np.int64))
    iat_min = (iat_mean * rng.uniform(0, 0.5, n)).astype(np.int64)
    pkt_min = np.minimum(fwd_min, np.where(nbwd > 0, bwd_min, fwd_min))
    pkt_max = np.maximum(fwd_max, bwd_max)
    pkt_mean = np.round((fwd_len + bwd_len) / np.maximum(npk + 1, 1), 6)
    pkt_std = np.round((pkt_max - pkt_min) * rng.uniform(0, 0.5, n), 6)
    zeros_i = np.zeros(n, np.int64)
    zeros_f = np.zeros(n, np.float64)
    hdr_fwd = nfwd * rng.choice(np.array([20, 32, 40]), n)
    hdr_bwd = nbwd * rng.choice(np.array([20, 32, 40]), n)
    init_fwd = np.where(looks_ddos, rng.choice(np.array([256, 29200, 8192]), n),
                        rng.integers(-1, 65536, n))
    init_bwd = np.where(looks_ddos, rng.choice(np.array([235, 229, -1]), n), rng.integers(-1, 65536, n))

    cols = {
        "Destination Port": port, "Flow Duration": dur, "Total Fwd Packets": nfwd,
        "Total Backward Packets": nbwd, "Total Length of Fwd Packets": fwd_len,
        "Total Length of Bwd Packets": bwd_len, "Fwd Packet Length Max": fwd_max,
        "Fwd Packet Length Min": fwd_min, "Fwd Packet Length Mean": fwd_mean,
        "Fwd Packet Length Std": fwd_std, "Bwd Packet Length Max": bwd_max,
        "Bwd Packet Length Min": bwd_min, "Bwd Packet Length Mean": bwd_mean,
        "Bwd Packet Length Std": bwd_std, "Flow Bytes/s": bytes_s, "Flow Packets/s": pkts_s,
        "Flow IAT Mean": iat_mean, "Flow IAT Std": iat_std, " Flow IAT Max": iat_max,
        "Flow IAT Min": iat_min, "Fwd IAT Total": dur, "Fwd IAT Mean": iat_mean,
        "Fwd IAT Std": iat_std, "Fwd IAT Max": iat_max, " Fwd IAT Min": iat_min,
        "Bwd IAT Total": np.where(nbwd > 1, dur, 0), "Bwd IAT Mean": np.where(nbwd > 1, iat_mean, 0.0),
        "Bwd IAT Std": zeros_f, "Bwd IAT Max": np.where(nbwd > 1, iat_max, 0),
        " Bwd IAT Min": np.where(nbwd > 1, iat_min, 0), "Fwd PSH Flags": zeros_i,
        "Bwd PSH Flags": zeros_i, "Fwd URG Flags": zeros_i, "Bwd URG Flags": zeros_i,
        "Fwd Header Length": hdr_fwd, "Bwd Header Length": hdr_bwd, "Fwd Packets/s": fwd_pkts_s,
        " Bwd Packets/s": bwd_pkts_s, " Min Packet Length": pkt_min, " Max Packet Length": pkt_max,
        "Packet Length Mean": pkt_mean, "Packet Length Std": pkt_std,
        "Packet Length Variance": np.round(pkt_std ** 2, 4),
        "FIN Flag Count": (rng.random(n) < 0.05).astype(np.int64),
        " SYN Flag Count": (rng.random(n) < 0.03).astype(np.int64),
        "RST Flag Count": zeros_i, "PSH Flag Count": (rng.random(n) < 0.4).astype(np.int64),
        "ACK Flag Count": (rng.random(n) < 0.5).astype(np.int64),
        "URG Flag Count": (rng.random(n) < 0.1).astype(np.int64), "CWE Flag Count": zeros_i,
        "ECE Flag Count": zeros_i, "Down/Up Ratio": (nbwd // nf_safe).astype(np.int64),
        "Average Packet Size": np.round(pkt_mean * 1.1, 6), "Avg Fwd Segment Size": fwd_mean,
        "Avg Bwd Segment Size": bwd_mean, "Fwd Header Length.1": hdr_fwd,
        "Fwd Avg Bytes/Bulk": zeros_i, "Fwd Avg Packets/Bulk": zeros_i, "Fwd Avg Bulk Rate": zeros_i,
        "Bwd Avg Bytes/Bulk": zeros_i, "Bwd Avg Packets/Bulk": zeros_i, "Bwd Avg Bulk Rate": zeros_i,
        "Subflow Fwd Packets": nfwd, "Subflow Fwd Bytes": fwd_len, "Subflow Bwd Packets": nbwd,
        "Subflow Bwd Bytes": bwd_len, "Init_Win_bytes_forward": init_fwd,
        "Init_Win_bytes_backward": init_bwd, "act_data_pkt_fwd": np.minimum(nfwd, 2),
        "min_seg_size_forward": rng.choice(np.array([20, 32]), n), "Active Mean": zeros_f,
        "Active Std": zeros_f, "Active Max": zeros_i, "Active Min": zeros_i, "Idle Mean": zeros_f,
        "Idle Std": zeros_f, "Idle Max": zeros_i, "Idle Min": zeros_i,
        "Label": np.where(is_ddos, "DDoS", "BENIGN"),
    }
    names = dedup_columns(CICIDS2017_COLUMNS)
    assert set(names) == set(cols), set(names) ^ set(cols)
    return pd.DataFrame({k: cols[k] for k in names})


def _lookalikes(rng, b, port, dur, nfwd, nbwd, fwd_max, fwd_min, fwd_len, bwd_len, bwd_max, bwd_min,
                frac=HARD_LOOKALIKE):
    """Turn ``frac`` of the BENIGN rows ``b`` into flood-shaped HTTP flows (in place)."""
    sel = b[rng.random(b.size) < frac]
    m = sel.size
    port[sel] = 80
    dur[sel] = np.exp(rng.uniform(np.log(5e2), np.log(1.2e8), m)).astype(np.int64)
    nfwd[sel] = rng.integers(1, 11, m)
    nbwd[sel] = np.where(rng.random(m) < 0.2, 0, rng.integers(2, 9, m))
    fwd_max[sel] = rng.choice(np.array([0, 6, 20, 31, 46]), m)
    fwd_min[sel] = 0
    fwd_len[sel] = np.minimum(fwd_max[sel] * rng.integers(1, 3, m), fwd_max[sel] * nfwd[sel])
    pay = np.where(rng.random(m) < 1.0 / 3.0, rng.choice(np.array([11595, 11601, 11607, 5840, 7300]), m),
                   rng.integers(2000, 14000, m))
    bwd_len[sel] = np.where(nbwd[sel] > 0, pay, 0)
    bwd_max[sel] = np.where(nbwd[sel] > 0, np.minimum(bwd_len[sel], 5840 + rng.integers(0, 2, m) * 1460), 0)
    bwd_min[sel] = 0


def write_csv(df: pd.DataFrame, path: str) -> None:
    """Write with the original (non-deduplicated) header and 'Infinity' spelling."""
    out = df.copy()
    out.columns = CICIDS2017_COLUMNS
    out.to_csv(path, index=False, na_rep="NaN", float_format=None)
