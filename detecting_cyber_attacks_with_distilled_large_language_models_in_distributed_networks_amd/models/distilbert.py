"""Arena-backed DistilBERT + ``DDoSClassifier`` (reference client1.py:53-65).

Public surface kept from the reference:
  * ``DDoSClassifier(local_model_path)`` with attributes ``.distilbert``,
    ``.dropout`` (p=0.3) and ``.classifier`` (Linear 768->2);
  * ``forward(input_ids, attention_mask) -> logits [B, 2]``;
  * ``state_dict()`` with the exact 102 fp32 keys / shapes / order of the
    reference checkpoint (``distilbert.embeddings.word_embeddings.weight`` ...
    ``classifier.bias``), loadable by ``load_state_dict``.

MI355X design: every parameter is a view into one flat fp32 arena (with a
bf16 shadow the kernels read and a flat fp32 grad arena the backward writes),
and ``impl="hip"`` runs the fused gfx950 kernels through three autograd node
types (ops/functional.py).  ``impl="torch"`` is the pure-PyTorch fp32 path used
on CPU (gloo plumbing, tests).  ``forward_loss`` fuses the head with the CE loss.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import torch
import torch.nn as nn

from ..ops import reference as R
from ..data.dataset import short_batch
from .arena import ParamArena


@dataclass
class DistilBertConfig:
    vocab_size: int = 30522
    dim: int = 768
    n_layers: int = 6
    n_heads: int = 12
    hidden_dim: int = 3072
    max_position_embeddings: int = 512
    dropout: float = 0.1
    attention_dropout: float = 0.1
    pad_token_id: int = 0
    layer_norm_eps: float = 1e-12
    initializer_range: float = 0.02


LAYER_KEYS = [  # HF registration (= state_dict) order inside a TransformerBlock
    ("attention.q_lin.weight", "w"), ("attention.q_lin.bias", "b"),
    ("attention.k_lin.weight", "w"), ("attention.k_lin.bias", "b"),
    ("attention.v_lin.weight", "w"), ("attention.v_lin.bias", "b"),
    ("attention.out_lin.weight", "w"), ("attention.out_lin.bias", "b"),
    ("sa_layer_norm.weight", "g"), ("sa_layer_norm.bias", "b"),
    ("ffn.lin1.weight", "w"), ("ffn.lin1.bias", "b"),
    ("ffn.lin2.weight", "w"), ("ffn.lin2.bias", "b"),
    ("output_layer_norm.weight", "g"), ("output_layer_norm.bias", "b"),
]


def gpu_shared() -> bool:
    """Whether this process shares its GPU with other ranks of the job (more local ranks than
    visible GPUs, e.g. ``FEDDDOS_BACKEND=gloo`` clients on a 1-GPU box)."""
    local = int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1)
    if local <= 1 or not torch.cuda.is_available():
        return False
    return local > torch.cuda.device_count()


def _layer_shapes(cfg: DistilBertConfig) -> Dict[str, Tuple[int, ...]]:
    D, F = cfg.dim, cfg.hidden_dim
    return {
        "attention.q_lin.weight": (D, D), "attention.q_lin.bias": (D,),
        "attention.k_lin.weight": (D, D), "attention.k_lin.bias": (D,),
        "attention.v_lin.weight": (D, D), "attention.v_lin.bias": (D,),
        "attention.out_lin.weight": (D, D), "attention.out_lin.bias": (D,),
        "sa_layer_norm.weight": (D,), "sa_layer_norm.bias": (D,),
        "ffn.lin1.weight": (F, D), "ffn.lin1.bias": (F,),
        "ffn.lin2.weight": (D, F), "ffn.lin2.bias": (D,),
        "output_layer_norm.weight": (D,), "output_layer_norm.bias": (D,),
    }


# Arena order: q/k/v weights then q/k/v biases contiguous (fused QKV views).
_ARENA_LAYER_ORDER = [
    "attention.q_lin.weight", "attention.k_lin.weight", "attention.v_lin.weight",
    "attention.q_lin.bias", "attention.k_lin.bias", "attention.v_lin.bias",
    "attention.out_lin.weight", "attention.out_lin.bias",
    "sa_layer_norm.weight", "sa_layer_norm.bias",
    "ffn.lin1.weight", "ffn.lin1.bias", "ffn.lin2.weight", "ffn.lin2.bias",
    "output_layer_norm.weight", "output_layer_norm.bias",
]


def encoder_specs(cfg: DistilBertConfig, prefix: str, token_types: int = 0) -> List[Tuple[str, Tuple[int, ...]]]:
    """token_types > 0: a BERT token-type table after the position table (models/bert.py)."""
    D = cfg.dim
    specs = [(f"{prefix}embeddings.word_embeddings.weight", (cfg.vocab_size, D)),
             (f"{prefix}embeddings.position_embeddings.weight", (cfg.max_position_embeddings, D))]
    if token_types:
        specs.append((f"{prefix}embeddings.token_type_embeddings.weight", (token_types, D)))
    specs += [(f"{prefix}embeddings.LayerNorm.weight", (D,)),
              (f"{prefix}embeddings.LayerNorm.bias", (D,))]
    shapes = _layer_shapes(cfg)
    for i in range(cfg.n_layers):
        for k in _ARENA_LAYER_ORDER:
            specs.append((f"{prefix}transformer.layer.{i}.{k}", shapes[k]))
    return specs


class _P(nn.Module):
    """Leaf module whose parameters are views into the arena."""

    def __init__(self, arena: ParamArena, prefix: str, names=("weight", "bias")):
        super().__init__()
        self._arena_keys = {}
        for n in names:
            key = prefix + n
            self._arena_keys[n] = key
            self.register_parameter(n, nn.Parameter(arena.view(key)))

    def rebind(self, arena: ParamArena):
        for n, key in self._arena_keys.items():
            p = getattr(self, n)
            p.data = arena.view(key)
            p.grad = arena.gview(key)


class _Embeddings(nn.Module):
    def __init__(self, arena, prefix, cfg):
        super().__init__()
        self.word_embeddings = _P(arena, prefix + "word_embeddings.", ("weight",))
        self.position_embeddings = _P(arena, prefix + "position_embeddings.", ("weight",))
        if prefix + "token_type_embeddings.weight" in arena.offsets:  # BERT teacher (HF registration order)
            self.token_type_embeddings = _P(arena, prefix + "token_type_embeddings.", ("weight",))
        self.LayerNorm = _P(arena, prefix + "LayerNorm.")
        self.dropout = nn.Dropout(cfg.dropout)


class _Attention(nn.Module):
    def __init__(self, arena, prefix, cfg):
        super().__init__()
        self.n_heads, self.dim = cfg.n_heads, cfg.dim
        self.dropout = nn.Dropout(cfg.attention_dropout)
        for n in ("q_lin", "k_lin", "v_lin", "out_lin"):
            setattr(self, n, _P(arena, f"{prefix}{n}."))


class _FFN(nn.Module):
    def __init__(self, arena, prefix, cfg):
        super().__init__()
        self.dropout = nn.Dropout(cfg.dropout)
        self.lin1 = _P(arena, prefix + "lin1.")
        self.lin2 = _P(arena, prefix + "lin2.")


class _Block(nn.Module):
    def __init__(self, arena, prefix, cfg):
        super().__init__()
        self.attention = _Attention(arena, prefix + "attention.", cfg)
        self.sa_layer_norm = _P(arena, prefix + "sa_layer_norm.")
        self.ffn = _FFN(arena, prefix + "ffn.", cfg)
        self.output_layer_norm = _P(arena, prefix + "output_layer_norm.")


class _Transformer(nn.Module):
    def __init__(self, arena, prefix, cfg):
        super().__init__()
        self.n_layers = cfg.n_layers
        self.layer = nn.ModuleList([_Block(arena, f"{prefix}layer.{i}.", cfg) for i in range(cfg.n_layers)])


class DistilBertEncoder(nn.Module):
    """Module tree with HF DistilBertModel's attribute names (state_dict parity)."""

    def __init__(self, arena: ParamArena, prefix: str, cfg: DistilBertConfig):
        super().__init__()
        self.config = cfg
        self.prefix = prefix
        self.embeddings = _Embeddings(arena, prefix + "embeddings.", cfg)
        self.transformer = _Transformer(arena, prefix + "transformer.", cfg)


# ---------------------------------------------------------------------------- init / loading
def init_encoder_(arena: ParamArena, prefix: str, cfg: DistilBertConfig, gen: torch.Generator):
    """HF DistilBERT _init_weights: Linear/Embedding ~ N(0, 0.02), bias 0, LN (1, 0), pad row 0."""
    for name, shape in arena.specs:
        if not name.startswith(prefix):
            continue
        v = arena.view(name)
        if name.endswith("LayerNorm.weight") or name.endswith("layer_norm.weight"):
            cpu = torch.ones(shape)
        elif name.endswith(".bias"):
            cpu = torch.zeros(shape)
        else:
            cpu = torch.randn(shape, generator=gen) * cfg.initializer_range
            if name.endswith("word_embeddings.weight"):
                cpu[cfg.pad_token_id] = 0
        v.copy_(cpu)


def load_hf_weights(arena: ParamArena, prefix: str, path: str) -> int:
    """Load an HF distilbert dir (model.safetensors or pytorch_model.bin) if present."""
    sd = None
    st = os.path.join(path, "model.safetensors")
    pt = os.path.join(path, "pytorch_model.bin")
    if os.path.exists(st):
        from safetensors.torch import load_file
        sd = load_file(st)
    elif os.path.exists(pt):
        sd = torch.load(pt, map_location="cpu", weights_only=True)
    if sd is None:
        return 0
    n = 0
    for k, v in sd.items():
        key = k if k.startswith(prefix) else prefix + k.removeprefix("distilbert.")
        if key in arena.offsets and tuple(v.shape) == arena.offsets[key][1]:
            arena.view(key).copy_(v.float())
            n += 1
    return n


# ---------------------------------------------------------------------------- classifier
class DDoSClassifier(nn.Module):
    """DistilBERT + Dropout(0.3) + Linear(768, 2) (client1.py:53-65)."""

    TOKEN_TYPES = 0  # DistilBERT has no token-type embeddings (the BERT teacher: 2)

    def __init__(self, local_model_path: Optional[str] = None, config: Optional[DistilBertConfig] = None,
                 device=None, impl: str = "auto", seed: int = 0, head_dropout: float = 0.3):
        super().__init__()
        cfg = config or DistilBertConfig()
        self.config = cfg
        device = torch.device(device) if device is not None else torch.device("cpu")
        specs = encoder_specs(cfg, "distilbert.", self.TOKEN_TYPES) + [("classifier.weight", (2, cfg.dim)),
                                                                        ("classifier.bias", (2,))]
        self.arena = ParamArena(specs, device="cpu", with_shadow=False)
        gen = torch.Generator().manual_seed(seed)
        init_encoder_(self.arena, "distilbert.", cfg, gen)
        bound = 1.0 / math.sqrt(cfg.dim)  # nn.Linear default init
        self.arena.view("classifier.weight").copy_(torch.rand(2, cfg.dim, generator=gen) * 2 * bound - bound)
        self.arena.view("classifier.bias").copy_(torch.rand(2, generator=gen) * 2 * bound - bound)
        self.loaded_pretrained = 0
        if local_model_path is not None and os.path.isdir(local_model_path):
            self.loaded_pretrained = load_hf_weights(self.arena, "distilbert.", local_model_path)
        self.distilbert = DistilBertEncoder(self.arena, "distilbert.", cfg)
        self.dropout = nn.Dropout(head_dropout)
        self.classifier = _P(self.arena, "classifier.")
        self.impl_request = impl
        # HIP path: only the word-embedding rows present in the batch carry a gradient
        # (emb_now flags); ArenaAdam skips the rest exactly.  Set False for a dense grad.
        self.sparse_word_grad = True
        # set by an overlapping optimizer (engine/optim.py): called per block during backward
        self.layer_grads_hook = None
        # (Removed after losing their A/B, logs in profiles/: the weight-gradient GEMMs on a side
        # stream -- 3.24 vs 3.20 ms/step, r1_ab_wgrad_side_stream.txt; per-step W^T copies for the
        # backward's dX GEMMs -- 1.7343 vs 1.7031 ms/step, r4_ab_dx_layouts.txt (the dX GEMMs read
        # W itself); the embedding backward + column-sum flush beside the dW launch -- neutral,
        # r2_ab_tail_overlap_groupm.txt.)
        # HIP path: grouped weight-gradient GEMMs (RunCtx.group_dw)
        self.group_dw = True
        # HIP path: every weight gradient of the step in one launch at the end of the backward
        # (RunCtx.dw_batch; needs no per-block gradient hook / weight-gradient side stream)
        self.batch_dw = os.environ.get("FD_BATCH_DW", "1") != "0"
        # optional fp32 [1] device tensor: the HIP head kernel adds every training step's mean
        # loss to it (RunCtx.loss_acc; bench.py reads one sum after a graph-replayed loop).  A
        # captured graph holds its address: keep it alive as long as that graph is replayed.
        self.loss_acc = None
        # HIP path: when the caller passes the batch's real-token count (DeviceLoader does,
        # from host-side lengths -- no sync), run the transformer blocks on the packed real
        # tokens only (~37 % of a seq128 CICIDS2017 batch is padding).  Rows are rounded up
        # to `pack_quantum` so a handful of shapes (HIP graphs) cover every batch.
        self.unpad = True
        # (a multiple of 64: the weight-gradient K steps; 64 rather than 128: -4 us per step in 4
        # interleaved 200-step pairs, profiles/r6_ab_pack_quantum.txt -- fewer padding rows, and the
        # CICIDS2017 batches still fall in 2-3 buckets)
        self.pack_quantum = int(os.environ.get("FD_PACK_QUANTUM", "64"))
        # HIP path: finalise all bias / LN-affine column sums of a backward in one launch
        self.defer_colsum = True
        # HIP path: reduce all split-K weight-gradient slabs of a backward in one launch
        self.defer_dw_reduce = True
        # HIP path: FFN lin1's bias gradient summed in the GELU' dX GEMM epilogue
        self.fuse_colsum = True
        # HIP path: the forward keeps the FFN activation g = gelu(u) for the backward (FD_REMAT_GELU=1:
        # the GELU' dX epilogue re-creates it instead -- round 1's win, -1.3 %, is now a loss: the
        # all-layer dW launch keeps every g live to the end anyway, and the epilogue's 16.5 MB write
        # per layer costs 11 us per step, profiles/r6_ab_remat_gelu.txt)
        self.remat_gelu = os.environ.get("FD_REMAT_GELU", "0") != "0"
        # HIP path: LayerNorm fused into the N = 768 GEMMs (RunCtx.fuse_ln; FD_FUSE_LN=0: the
        # separate LN kernels).  Hidden sizes the fused epilogue does not cover fall back.
        # Its row blocks wait on each other's statistics, so every tile of a launch must be resident
        # at once: off when other processes share this GPU (e.g. several gloo clients on one card),
        # whose kernels could hold CUs through a rendezvous (a timeout is fatal: check_ln_error).
        self.fuse_ln = os.environ.get("FD_FUSE_LN", "1") != "0" and not gpu_shared()
        # HIP path (with batch_dw): the per-block qkv-bias column-sum partials in one launch at the
        # end of the backward (RunCtx.colsum_pending; FD_BATCH_COLSUM=0: one launch per block)
        self.batch_colsum = os.environ.get("FD_BATCH_COLSUM", "1") != "0"
        # HIP path (packed step): the Adam step / dropout seed counters are advanced by the packing
        # launch instead of a kernel of their own (FD_FOLD_STEP=0: separate launch)
        self.fold_step_counters = os.environ.get("FD_FOLD_STEP", "1") != "0"
        # HIP path: the last block runs its out-proj / FFN / LayerNorms on the [CLS] rows only
        # (exact: no other row of its output reaches the loss; FD_PRUNE_LAST=0: every row)
        self.prune_last = os.environ.get("FD_PRUNE_LAST", "1") != "0"
        # optimizer that applies Adam inside the weight-gradient GEMM epilogues; set only for
        # the duration of a training step (engine/train.py fused_adam_scope)
        self.fused_opt = None
        # optimizer of the running training step (same scope): its step counter is advanced
        # by the forward's dropout-seed launch
        self.step_opt = None
        self.torch_counter = 0
        self._grad_token = None
        self._synced_version = -1
        self._hip_cache = None
        self.to(device)

    # -------------------------------------------------------------- device management
    def _apply(self, fn, recurse=True):
        probe = fn(self.arena.master[:1])
        if probe.dtype != torch.float32:
            raise TypeError("DDoSClassifier keeps fp32 master weights; compute dtype is the bf16 shadow")
        self.arena.to(probe.device)
        for m in self.modules():
            if isinstance(m, _P):
                m.rebind(self.arena)
        dev = probe.device
        self.rng = torch.zeros(1, dtype=torch.int32, device=dev)
        # Sparse word-embedding gradient (HIP path): rows valid this step / rows with Adam state.
        V = self.config.vocab_size
        self.emb_now = torch.zeros(V, dtype=torch.uint8, device=dev) if dev.type == "cuda" else None
        self.emb_ever = torch.zeros(V, dtype=torch.uint8, device=dev) if dev.type == "cuda" else None
        self._grad_token = torch.zeros((), device=dev, requires_grad=True)
        self._hip_cache = None
        self._synced_version = -1
        return self

    @property
    def device(self) -> torch.device:
        return self.arena.device

    @property
    def impl(self) -> str:
        if self.impl_request == "auto":
            return "hip" if self.arena.device.type == "cuda" else "torch"
        if self.impl_request == "hip" and self.arena.device.type != "cuda":
            raise RuntimeError("impl='hip' needs the model on a GPU")
        return self.impl_request

    def layer_span(self, i: int) -> Tuple[int, int]:
        """(arena offset, length) of transformer block i's parameters (contiguous, 64-aligned)."""
        pre = f"distilbert.transformer.layer.{i}."
        offs = [(o, math.prod(sh)) for nm, (o, sh) in self.arena.offsets.items() if nm.startswith(pre)]
        lo = min(o for o, _ in offs)
        hi = max(o + n for o, n in offs)
        return lo, (hi - lo + 63) // 64 * 64

    def word_embedding_span(self):
        """(arena offset, rows, row_len) of the word-embedding table."""
        off, shape = self.arena.offsets["distilbert.embeddings.word_embeddings.weight"]
        return off, shape[0], shape[1]

    def dense_grad(self, name: str) -> torch.Tensor:
        """Gradient of ``name`` with the sparse word-embedding rows materialised (zeros elsewhere)."""
        g = self.arena.gview(name)
        if name.endswith("word_embeddings.weight") and self.emb_now is not None and self.sparse_word_grad \
                and self.impl == "hip":
            g = g * self.emb_now.to(g.dtype)[:, None]
        return g

    def zero_grad(self, set_to_none: bool = False):
        # hip: first-write kernels make zeroing unnecessary; torch: autograd accumulates into the arena.
        self.arena.zero_grad(zero_buffer=(self.impl == "torch"))
        for m in self.modules():
            if isinstance(m, _P):
                for n, key in m._arena_keys.items():
                    getattr(m, n).grad = self.arena.gview(key)

    def _param_version(self) -> int:
        # Parameters keep their own version counters (p.data = view), so sum them:
        # any in-place update (load_state_dict, torch.optim, FedAvg) changes it.
        return self.arena.master._version + sum(p._version for p in self.parameters())

    def sync_shadow(self, force: bool = False):
        """Refresh the bf16 compute shadow if the fp32 masters changed outside our Adam."""
        v = self._param_version()
        if force or v != self._synced_version:
            self.arena.sync_shadow()
            self._synced_version = self._param_version()

    def mark_shadow_synced(self):
        """The shadow was rewritten outside ``sync_shadow`` (an Adam step, FedAvg's scale_cast)."""
        self._synced_version = self._param_version()

    def prepare_replay(self):
        """Eager state a captured training step does not refresh by itself, brought up to date
        before every replay and capture (``GraphedTrainStep``, step_fn.prepare): the bf16 shadow the
        kernels read, after an out-of-band write of the fp32 masters (``load_state_dict``, a torch
        optimizer, ...).  A captured forward holds no ``sync_shadow`` of its own, so without this a
        replay after a checkpoint load would train the pre-load weights.  (Writers that keep the
        shadow current themselves -- the Adam kernels, FedAvg's scale_cast -- call
        ``mark_shadow_synced``; the check is a host-side version compare.)"""
        self.sync_shadow()

    # -------------------------------------------------------------- HIP handles
    def _hip_handles(self):
        if self._hip_cache is not None:
            return self._hip_cache
        from ..ops.functional import GradSink
        A = self.arena
        pre = "distilbert."
        tt_name = pre + "embeddings.token_type_embeddings.weight"
        if tt_name in A.offsets:
            # BERT teacher, token_type_ids all 0: type row 0 folded into the position table the
            # kernels read (refreshed every forward, _run_hip); its gradient is the column sum
            # of the position gradient (EmbeddingFn)
            pos_tab = torch.empty_like(A.sview(pre + "embeddings.position_embeddings.weight"))
        else:
            pos_tab = A.sview(pre + "embeddings.position_embeddings.weight")
        emb = {
            "word": A.sview(pre + "embeddings.word_embeddings.weight"),
            "pos": pos_tab,
            "ln_w": A.view(pre + "embeddings.LayerNorm.weight"),
            "ln_b": A.view(pre + "embeddings.LayerNorm.bias"),
            "sinks": {
                "word": GradSink(A, pre + "embeddings.word_embeddings.weight"),
                "pos": GradSink(A, pre + "embeddings.position_embeddings.weight"),
                "ln_w": GradSink(A, pre + "embeddings.LayerNorm.weight"),
                "ln_b": GradSink(A, pre + "embeddings.LayerNorm.bias"),
                "flags": (self.emb_now, self.emb_ever) if self.sparse_word_grad else None,
            },
        }
        if tt_name in A.offsets:
            emb["sinks"]["type"] = GradSink(A, tt_name)
        layers = []
        for i in range(self.config.n_layers):
            lp = f"{pre}transformer.layer.{i}."
            qkv_w = [lp + f"attention.{n}_lin.weight" for n in "qkv"]
            qkv_b = [lp + f"attention.{n}_lin.bias" for n in "qkv"]
            names = {
                "o_w": lp + "attention.out_lin.weight", "o_b": lp + "attention.out_lin.bias",
                "ln1_w": lp + "sa_layer_norm.weight", "ln1_b": lp + "sa_layer_norm.bias",
                "l1_w": lp + "ffn.lin1.weight", "l1_b": lp + "ffn.lin1.bias",
                "l2_w": lp + "ffn.lin2.weight", "l2_b": lp + "ffn.lin2.bias",
                "ln2_w": lp + "output_layer_norm.weight", "ln2_b": lp + "output_layer_norm.bias",
            }
            L = {"qkv_w": A.span(qkv_w, "shadow"), "qkv_b": A.span(qkv_b, "master")}
            sinks = {"qkv_w": _SpanSink(A, qkv_w), "qkv_b": _SpanSink(A, qkv_b)}
            for k, nm in names.items():
                L[k] = A.sview(nm) if k.endswith("_w") and not k.startswith("ln") else A.view(nm)
                sinks[k] = GradSink(A, nm)
            L["sinks"] = sinks
            layers.append(L)
        head = {"w": A.view("classifier.weight"), "b": A.view("classifier.bias"),
                "sinks": {"w": GradSink(A, "classifier.weight"), "b": GradSink(A, "classifier.bias")}}
        self._hip_cache = (emb, layers, head)
        return self._hip_cache

    # -------------------------------------------------------------- forward
    def forward(self, input_ids: torch.Tensor, attention_mask: torch.Tensor,
                tokens: Optional[int] = None) -> torch.Tensor:
        return self._run(input_ids, attention_mask, None, tokens)[1]

    def forward_loss(self, input_ids, attention_mask, labels,
                     tokens: Optional[int] = None, kd=None,
                     unit_backward: bool = False) -> Tuple[torch.Tensor, torch.Tensor]:
        """(mean CE loss, logits) with the head and the loss fused (one kernel).

        tokens: number of real (mask = 1) tokens in the batch, if the caller knows it
        without a device sync -- enables the unpadded HIP path (same math: padding
        positions never reach a real token or the loss).
        kd = (teacher logits [B, 2], temperature, alpha): the loss is the distillation loss
        (models/bert.py ``kd_loss``), fused into the same head kernel on the HIP path.
        unit_backward: the caller promises ``loss.backward(ops.kernels.unit_grad(device))`` (the
        training step functions of engine/train.py): the [CLS]-pruned HIP step then runs the head's
        backward and the last block's output-LayerNorm backward inside the head's forward launch
        (ops/kernels.py head_ln_bwd; a backward seeded with anything else raises)."""
        return self._run(input_ids, attention_mask, labels, tokens, kd, unit_backward)

    def _run(self, input_ids, attention_mask, labels, tokens=None, kd=None, unit_backward=False):
        if self.impl == "hip":
            return self._run_hip(input_ids, attention_mask, labels, tokens, kd, unit_backward)
        loss, logits = self._run_torch(input_ids, attention_mask, labels if kd is None else None)
        if kd is not None and labels is not None:
            from .bert import kd_loss
            loss = kd_loss(logits, kd[0], labels, kd[1], kd[2])
        return loss, logits

    def packed_rows(self, tokens: int, B: int, S: int) -> int:
        """Row count of the packed layout for a batch with ``tokens`` real tokens."""
        q = self.pack_quantum
        return min(B * S, (int(tokens) + q - 1) // q * q)

    def _run_hip(self, ids, mask, labels, tokens=None, kd=None, unit_backward=False):
        from ..ops import kernels as K
        from ..ops.functional import EmbeddingFn, HeadFn, LayerFn, RunCtx
        self.sync_shadow()
        B, S = ids.shape
        if S % 64:
            pad = 64 - S % 64
            ids = torch.nn.functional.pad(ids, (0, pad))
            mask = torch.nn.functional.pad(mask, (0, pad))
            S += pad
        emb, layers, head = self._hip_handles()
        cfg = self.config
        if self.TOKEN_TYPES:
            A = self.arena
            emb["pos"].copy_(A.view("distilbert.embeddings.position_embeddings.weight")
                             + A.view("distilbert.embeddings.token_type_embeddings.weight")[0])
        grad = torch.is_grad_enabled()
        packed = tokens is not None and self.unpad and self.packed_rows(tokens, B, S) < B * S
        # varlen attention masks keys by sequence length; the padded path needs the additive bias
        kbias = self._no_bias() if packed else K.mask_bias(mask)
        rc = RunCtx(B=B, S=S, H=cfg.n_heads, kbias=kbias, seed=self.rng, training=self.training,
                    eps=cfg.layer_norm_eps, p_hidden=cfg.dropout, p_attn=cfg.attention_dropout, p_head=self.dropout.p,
                    on_layer_grads=self.layer_grads_hook if grad else None, group_dw=self.group_dw,
                    loss_acc=getattr(self, "loss_acc", None), unit_backward=bool(unit_backward and grad))
        if grad and self.defer_colsum and self.layer_grads_hook is None:
            rc.colsum_jobs = []  # (a per-block hook needs each block's grads final at once)
        if grad and self.defer_dw_reduce and self.layer_grads_hook is None:
            rc.dw_jobs = []
        if grad and self.batch_dw and self.layer_grads_hook is None:
            rc.dw_batch = []
            if rc.colsum_jobs is not None and self.batch_colsum:
                rc.colsum_pending = []
        rc.fuse_colsum = self.fuse_colsum
        rc.attn_short = packed and short_batch(tokens, S)
        rc.qkv_ws = [L["qkv_w"] for L in layers]
        rc.remat_gelu = self.remat_gelu
        rc.fuse_ln = self.fuse_ln and cfg.dim % 64 == 0 and cfg.dim <= 2048
        # a data-parallel client's gradient exchange overlaps the backward (parallel/dp.py GradSync
        # sets collectives_in_backward): no LayerNorm-fused backward GEMM beside RCCL's kernels
        rc.fuse_ln_bwd = rc.fuse_ln and K.ln_fusable(
            1, cfg.dim, concurrent_collectives=bool(grad and getattr(self, "collectives_in_backward", False)))
        if grad and self.training and self.fused_opt is not None and self.layer_grads_hook is None:
            # (the per-layer grouped dW path applies it only where the dX GEMMs read W^T copies taken
            # before the step; the all-layer dW launch runs after every dX GEMM of the backward)
            rc.fused_adam = self.fused_opt
        plan = self._prune_plan(rc, layers, grad)
        # packed step: the counters ride on the packing launch (no kernel of their own)
        incs = [] if packed and self.fold_step_counters else None
        if self.training:
            if grad and self.step_opt is not None:
                self.step_opt._begin(seed=self.rng, defer=incs)  # Adam step + dropout seed: one launch
            elif incs is not None:
                incs.append((None, self.rng))
            else:
                K.step_inc(None, self.rng)
        token = self._grad_token if torch.is_grad_enabled() else None
        if packed:
            # Unpadded step: only the real tokens (sequence-contiguous, filler rows at the end)
            # are embedded and run through the blocks; varlen attention over cu; positions and
            # dropout follow the padded row (same masks as the padded path); the head reads
            # row cu[b] for sequence b's [CLS].  Filler rows act as padded row 0: finite, and
            # their gradient is exactly 0 (they reach neither a real token nor the loss).
            # The layout (row map, sequence starts, packed ids) is one kernel (ops/packing).
            incs = incs or []
            st_inc = next((a for a, _ in incs if a is not None), None)
            sd_inc = next((b for _, b in incs if b is not None), None)
            if len([a for a, _ in incs if a is not None]) > 1 or len([b for _, b in incs if b is not None]) > 1:
                raise RuntimeError("a counter deferred twice in one forward")
            rc.row_map, rc.cu, ids = K.pack(mask, ids, self.packed_rows(tokens, B, S), step=st_inc, seed=sd_inc,
                                            cls_rows=plan[4] if plan is not None else None,
                                            cls_rmap=plan[5] if plan is not None else None)
        x = EmbeddingFn.apply(token, ids, emb["word"], emb["pos"], emb["ln_w"], emb["ln_b"], emb["sinks"], rc)
        self._setup_prune(rc, plan, len(layers), packed)
        if (labels is not None and grad and self.training and rc.unit_backward and rc.prune_idx >= 0
                and rc.colsum_jobs is not None and rc.head_rows is not None):
            # (the pruned block may run the head inside its output-LayerNorm launch: ops/functional.py)
            rc.head_req = (head, labels.to(torch.int64), kd)
        for i, L in enumerate(layers):
            x = LayerFn.apply(x, L, rc, i)
        if labels is not None:
            loss, logits = HeadFn.apply(x, head["w"], head["b"], head["sinks"], rc, labels.to(torch.int64), kd)
            return loss, logits
        logits, _ = HeadFn.apply(x, head["w"], head["b"], head["sinks"], rc, None)
        return None, logits

    def _prune_plan(self, rc, layers, grad: bool):
        """Last-block [CLS] pruning (RunCtx.prune_idx; ops/functional.py LayerFn._forward_pruned):
        exact -- the dropped rows reach neither the loss nor any gradient.  Needs the fused
        LayerNorm path and, for a training step, the all-layer dW launch (the pruned block's
        out-proj / FFN weight gradients join it with K = Bp rows).  Returns the
        per-shape index buffers (the packing launch fills the packed [CLS] rows), or None."""
        from ..ops import kernels as K
        B, S, D = rc.B, rc.S, self.config.dim
        Bp = (B + 63) // 64 * 64
        if not (self.prune_last and rc.fuse_ln and layers and K.ln_fusable(Bp, D) and Bp <= rc.B * rc.S):
            return None
        if grad and rc.dw_batch is None:
            return None
        dev = self.arena.device
        key = (B, S, Bp, str(dev))
        # One buffer set per batch shape, kept for the model's lifetime: HIP graphs captured for one
        # shape (the bs16 eval forward) hold these addresses while another shape (the bs32 train
        # step) runs -- replacing the set would free memory a later replay reads and writes
        # (round 4: a second client's eval replay faulted on the first client's freed buffers).
        caches = self.__dict__.setdefault("_prune_caches", {})
        cache = caches.get(key)
        if cache is None:
            rmap = torch.zeros(Bp, dtype=torch.int32, device=dev)
            rmap[:B] = torch.arange(B, dtype=torch.int32, device=dev) * S
            padded_rows = rmap.to(torch.int64)  # padded layout: sequence b's [CLS] is row b * S
            # (packed: the packing launch fills the kept rows and their dropout-hash rows)
            cache = (key, rmap, padded_rows, torch.arange(B, dtype=torch.int32, device=dev),
                     torch.zeros(Bp, dtype=torch.int64, device=dev), torch.zeros(Bp, dtype=torch.int32, device=dev))
            caches[key] = cache
        return cache

    @staticmethod
    def _setup_prune(rc, plan, n_layers: int, packed: bool):
        if plan is None:
            return
        _, rmap, padded_rows, head_rows, packed_rows, packed_rmap = plan
        # packed: rows cu[b] and their padded rows (written by the packing launch); filler rows ->
        # row 0 (a finite row)
        rc.cls_rows = packed_rows if packed else padded_rows
        rc.cls_rmap = packed_rmap if packed else rmap
        rc.head_rows, rc.prune_idx = head_rows, n_layers - 1

    def _no_bias(self) -> torch.Tensor:
        """Placeholder key-bias tensor for the varlen path (the kernels do not read it)."""
        t = getattr(self, "_nobias", None)
        if t is None or t.device != self.arena.device:
            t = torch.zeros(1, dtype=torch.float32, device=self.arena.device)
            self._nobias = t
        return t

    def _run_torch(self, ids, mask, labels):
        cfg = self.config
        tr = self.training
        counter = None
        if tr:
            self.torch_counter += 1
            counter = self.torch_counter
        B, S = ids.shape
        e = self.distilbert.embeddings
        pos = e.position_embeddings.weight
        if hasattr(e, "token_type_embeddings"):  # BERT teacher: token_type_ids all 0
            pos = pos + e.token_type_embeddings.weight[0]
        x = R.embedding_ref(ids, e.word_embeddings.weight, pos, e.LayerNorm.weight,
                            e.LayerNorm.bias, cfg.layer_norm_eps, cfg.dropout if tr else 0.0, counter, 1)
        for i, blk in enumerate(self.distilbert.transformer.layer):
            a = blk.attention
            P = {
                "qkv_w": torch.cat([a.q_lin.weight, a.k_lin.weight, a.v_lin.weight]),
                "qkv_b": torch.cat([a.q_lin.bias, a.k_lin.bias, a.v_lin.bias]),
                "o_w": a.out_lin.weight, "o_b": a.out_lin.bias,
                "ln1_w": blk.sa_layer_norm.weight, "ln1_b": blk.sa_layer_norm.bias,
                "l1_w": blk.ffn.lin1.weight, "l1_b": blk.ffn.lin1.bias,
                "l2_w": blk.ffn.lin2.weight, "l2_b": blk.ffn.lin2.bias,
                "ln2_w": blk.output_layer_norm.weight, "ln2_b": blk.output_layer_norm.bias,
            }
            x = R.layer_ref(x, P, B, S, cfg.n_heads, mask, cfg.layer_norm_eps,
                            cfg.attention_dropout if tr else 0.0, cfg.dropout if tr else 0.0, counter,
                            16 + 4 * i, 17 + 4 * i)
        logits = R.head_ref(x, B, S, self.classifier.weight, self.classifier.bias, self.dropout.p if tr else 0.0,
                            counter, 2)
        if labels is None:
            return None, logits
        return torch.nn.functional.cross_entropy(logits, labels), logits


class _SpanSink:
    """GradSink over a fused span (q/k/v) -- the three names are written together."""

    def __init__(self, arena, names):
        self.arena, self.names = arena, list(names)

    @property
    def buf(self):
        return self.arena.span(self.names, "grad")

    def accumulate(self) -> bool:
        acc = False
        for n in self.names:
            acc = self.arena.mark_written(n)
        return acc


def reference_state_dict_keys(cfg: Optional[DistilBertConfig] = None) -> List[str]:
    """The 102 keys of the reference checkpoint, in order."""
    cfg = cfg or DistilBertConfig()
    keys = ["distilbert.embeddings.word_embeddings.weight", "distilbert.embeddings.position_embeddings.weight",
            "distilbert.embeddings.LayerNorm.weight", "distilbert.embeddings.LayerNorm.bias"]
    for i in range(cfg.n_layers):
        keys += [f"distilbert.transformer.layer.{i}.{k}" for k, _ in LAYER_KEYS]
    return keys + ["classifier.weight", "classifier.bias"]
