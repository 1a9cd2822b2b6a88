"""MI355X-native federated DistilBERT DDoS detection framework.

Capabilities mirror the reference scripts (client1.py / client2.py / server.py:
one-round, two-client FedAvg of a DistilBERT + Dropout(0.3) + Linear(768, 2)
``DDoSClassifier`` on CICIDS2017 flows rendered as English text) but the design
is MI355X-first:

* every GPU is one federated client (one process per GPU, ``torch.distributed``
  over RCCL/xGMI); FedAvg is a single all-reduce over a flat fp32 parameter arena
  instead of pickle+gzip over TCP (reference server.py:67-114);
* the DistilBERT hot path runs on hand-written gfx950 HIP kernels (MFMA GEMMs
  with fused epilogues, fused attention, residual+LayerNorm, embedding, CE head,
  single-launch Adam) -- see ``ops/`` and ``csrc/kernels``;
* the tokenizer and featuriser are native C++ (``csrc/text``).

Sub-packages: ``data`` (synthetic CICIDS2017, featuriser, tokenizer, datasets),
``models`` (arena-backed DistilBERT/BERT, pure-torch reference), ``ops`` (HIP
kernel bindings + autograd), ``engine`` (train/eval, HIP-graph step),
``parallel`` (comm, FedAvg, launcher, TCP compat transport), ``fed``
(client/server round orchestration), ``utils`` (logging, metrics, plots,
checkpoints, timers, fault injection, profiling).
"""

__version__ = "0.1.0"

from .config import FedConfig  # noqa: F401
