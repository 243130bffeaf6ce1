"""Module trees with the reference's parameter names, executed by the native engines.

* `ResNet50`  — torchvision.models.resnet50 topology (v1.5) so `Resnet50TSM.base_model` state-dict
  keys match (`conv1.weight`, `layer1.0.conv1.net.weight` once TSM-wrapped, `bn*.running_mean`, ...).
* `BertModel` — HF transformers BertModel names (`embeddings.word_embeddings.weight`,
  `encoder.layer.N.attention.self.query.weight`, `pooler.dense.weight`, ...), built from a config
  (the reference's `from_pretrained('bert-base-uncased')` needs the network; a local checkpoint
  can be loaded with load_state_dict).
* `NativeRoot` — mixin owning the flat parameter buffers and the compute precision.
"""
import math

import torch
from torch import nn

from . import flat as flatmod
from . import ops


# ============================================================================ native root
class NativeRoot:
    """Mixin for modules whose forward runs on libvcg_hip.

    precision: "fp32" (parity mode; f32-input MFMA) or "bf16" (bf16 activations and MFMA operands,
    fp32 accumulation / statistics / master weights)."""

    _vcg_precision = "fp32"

    @property
    def precision(self):
        return self._vcg_precision

    @precision.setter
    def precision(self, value):
        if value not in ("fp32", "bf16"):
            raise ValueError("precision must be 'fp32' or 'bf16'")
        for m in self.modules():
            if isinstance(m, NativeRoot):
                object.__setattr__(m, "_vcg_precision", value)

    def compute_dtype(self):
        return ops.torch_dtype(self.precision)

    def native_flat(self):
        params = list(self.parameters())
        if not params:
            raise RuntimeError("module has no parameters")
        dev = params[0].device
        if dev.type != "cuda":
            raise RuntimeError(
                f"{type(self).__name__}: the native MI355X path needs the module on the GPU (model.to('cuda')); "
                "there is no CPU fallback")
        dt = self.compute_dtype()
        want_shadow = None if dt == torch.float32 else dt
        f = getattr(self, "_vcg_flat", None)
        ok = (f is not None and f.device == dev and f.shadow_dtype == want_shadow and len(f.params) >= len(params)
              and all(id(p) in f.index for p in (params[0], params[-1])) and f.intact())
        if not ok:
            named = list(self.named_parameters())
            f = flatmod.FlatParams(named, dev, shadow_dtype=want_shadow, order=_flat_order([n for n, _ in named]))
            for m in self.modules():
                object.__setattr__(m, "_vcg_flat", f)
            self._bind_bn_counters(dev)
        f.refresh_shadow()
        return f

    # one int64 buffer for every BatchNorm's num_batches_tracked -> one increment per step
    def _bind_bn_counters(self, dev):
        bns = [m for m in self.modules() if isinstance(m, nn.BatchNorm2d) and m.num_batches_tracked is not None]
        if not bns:
            object.__setattr__(self, "_vcg_bn_counter", None)
            return
        buf = torch.stack([b.num_batches_tracked.detach().to(dev) for b in bns]).reshape(-1)
        for i, b in enumerate(bns):
            b._buffers["num_batches_tracked"] = buf[i]
        object.__setattr__(self, "_vcg_bn_counter", (buf, bns))

    def _bump_bn_counters(self):
        c = getattr(self, "_vcg_bn_counter", None)
        if c is None:
            return
        buf, bns = c
        if all(b._buffers.get("num_batches_tracked") is not None and
               b.num_batches_tracked.data_ptr() == buf[i].data_ptr() for i, b in enumerate(bns)):
            flags = [b.training and b.track_running_stats for b in bns]
            if all(flags):
                buf.add_(1)
                return
        for b in bns:
            if b.training and b.track_running_stats and b.num_batches_tracked is not None:
                b.num_batches_tracked.add_(1)

    def zero_grad(self, set_to_none=True):  # noqa: D401 - keeps grads as flat views
        f = getattr(self, "_vcg_flat", None)
        if f is not None and f.intact():
            f.zero_grad()
        else:
            super().zero_grad(set_to_none=set_to_none)

    def _anchor(self, dev):
        a = getattr(self, "_vcg_anchor", None)
        if a is None or a.device != dev:
            a = torch.zeros(0, device=dev, requires_grad=True)
            object.__setattr__(self, "_vcg_anchor", a)
        return a


def _flat_order(names):
    """Layout order: keep module order but put each BERT layer's query/key/value weights (and
    biases) back to back so the fused QKV GEMM reads one [3H, H] view."""
    out, seen = [], set()
    for n in names:
        if n in seen:
            continue
        if n.endswith("attention.self.query.weight"):
            pre = n[: -len("query.weight")]
            grp = [pre + "query.weight", pre + "key.weight", pre + "value.weight",
                   pre + "query.bias", pre + "key.bias", pre + "value.bias"]
            for g in grp:
                if g in names and g not in seen:
                    out.append(g)
                    seen.add(g)
            continue
        out.append(n)
        seen.add(n)
    return out


def new_seed():
    return int(torch.randint(0, 2 ** 62, (1,)).item())


# ============================================================================ ResNet-50
class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None):
        super().__init__()
        self.conv1 = nn.Conv2d(inplanes, planes, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(planes)
        self.conv2 = nn.Conv2d(planes, planes, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(planes)
        self.conv3 = nn.Conv2d(planes, planes * 4, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(planes * 4)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample
        self.stride = stride


class Identity(nn.Module):
    def forward(self, x):
        return x


class ResNet50(NativeRoot, nn.Module):
    """torchvision resnet50 topology; forward(x [N,3,H,W] fp32) -> [N, 2048] (fc = Identity)."""

    def __init__(self, num_classes=1000):
        super().__init__()
        self.inplanes = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, 2, 1)
        self.layer1 = self._make_layer(64, 3)
        self.layer2 = self._make_layer(128, 4, stride=2)
        self.layer3 = self._make_layer(256, 6, stride=2)
        self.layer4 = self._make_layer(512, 3, stride=2)
        self.avgpool = nn.AdaptiveAvgPool2d((1, 1))
        self.fc = nn.Linear(2048, num_classes)
        for m in self.modules():  # torchvision init
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def _make_layer(self, planes, blocks, stride=1):
        downsample = None
        if stride != 1 or self.inplanes != planes * 4:
            downsample = nn.Sequential(nn.Conv2d(self.inplanes, planes * 4, 1, stride=stride, bias=False),
                                       nn.BatchNorm2d(planes * 4))
        layers = [Bottleneck(self.inplanes, planes, stride, downsample)]
        self.inplanes = planes * 4
        for _ in range(1, blocks):
            layers.append(Bottleneck(self.inplanes, planes))
        return nn.Sequential(*layers)

    def forward(self, x):
        if not isinstance(self.fc, Identity):
            raise RuntimeError("native ResNet50 implements the fc=Identity trunk (Resnet50TSM / TwoStream usage)")
        from .functions import TrunkFn
        from .trunk import ResNetTrunk
        self.native_flat()
        need_grad = torch.is_grad_enabled()
        if self.training:
            self._bump_bn_counters()
        eng = ResNetTrunk(self, self.compute_dtype())
        return TrunkFn.apply(x.float().contiguous(), self._anchor(x.device), eng, need_grad, None)


# ============================================================================ BERT
class BertConfig:
    """The subset of transformers.BertConfig the encoder uses (bert-base-uncased defaults)."""

    def __init__(self, vocab_size=30522, hidden_size=768, num_hidden_layers=12, num_attention_heads=12,
                 intermediate_size=3072, hidden_dropout_prob=0.1, attention_probs_dropout_prob=0.1,
                 max_position_embeddings=512, type_vocab_size=2, layer_norm_eps=1e-12, pad_token_id=0,
                 initializer_range=0.02, output_attentions=False, **kwargs):
        self.vocab_size = vocab_size
        self.hidden_size = hidden_size
        self.num_hidden_layers = num_hidden_layers
        self.num_attention_heads = num_attention_heads
        self.intermediate_size = intermediate_size
        self.hidden_dropout_prob = hidden_dropout_prob
        self.attention_probs_dropout_prob = attention_probs_dropout_prob
        self.max_position_embeddings = max_position_embeddings
        self.type_vocab_size = type_vocab_size
        self.layer_norm_eps = layer_norm_eps
        self.pad_token_id = pad_token_id
        self.initializer_range = initializer_range
        self.output_attentions = output_attentions
        for k, v in kwargs.items():
            setattr(self, k, v)


class _Embeddings(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.word_embeddings = nn.Embedding(c.vocab_size, c.hidden_size, padding_idx=c.pad_token_id)
        self.position_embeddings = nn.Embedding(c.max_position_embeddings, c.hidden_size)
        self.token_type_embeddings = nn.Embedding(c.type_vocab_size, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class _SelfAttn(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.query = nn.Linear(c.hidden_size, c.hidden_size)
        self.key = nn.Linear(c.hidden_size, c.hidden_size)
        self.value = nn.Linear(c.hidden_size, c.hidden_size)
        self.dropout = nn.Dropout(c.attention_probs_dropout_prob)


class _SelfOut(nn.Module):
    def __init__(self, c, din):
        super().__init__()
        self.dense = nn.Linear(din, c.hidden_size)
        self.LayerNorm = nn.LayerNorm(c.hidden_size, eps=c.layer_norm_eps)
        self.dropout = nn.Dropout(c.hidden_dropout_prob)


class _Attention(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.self = _SelfAttn(c)
        self.output = _SelfOut(c, c.hidden_size)


class _Intermediate(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.intermediate_size)


class _Layer(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.attention = _Attention(c)
        self.intermediate = _Intermediate(c)
        self.output = _SelfOut(c, c.intermediate_size)


class _Encoder(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.layer = nn.ModuleList([_Layer(c) for _ in range(c.num_hidden_layers)])


class _Pooler(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.dense = nn.Linear(c.hidden_size, c.hidden_size)


class BertOutput:
    """Subset of transformers' BaseModelOutputWithPoolingAndCrossAttentions."""

    def __init__(self, last_hidden_state, pooler_output):
        self.last_hidden_state = last_hidden_state
        self.pooler_output = pooler_output
        self.attentions = None

    def __getitem__(self, i):
        return (self.last_hidden_state, self.pooler_output)[i]


class BertModel(NativeRoot, nn.Module):
    def __init__(self, config=None, add_pooling_layer=True):
        super().__init__()
        self.config = config if config is not None else BertConfig()
        c = self.config
        self.embeddings = _Embeddings(c)
        self.encoder = _Encoder(c)
        self.pooler = _Pooler(c) if add_pooling_layer else None
        self._init_weights()

    def _init_weights(self):
        std = self.config.initializer_range
        for m in self.modules():
            if isinstance(m, nn.Linear):
                nn.init.normal_(m.weight, 0.0, std)
                nn.init.zeros_(m.bias)
            elif isinstance(m, nn.Embedding):
                nn.init.normal_(m.weight, 0.0, std)
                if m.padding_idx is not None:
                    with torch.no_grad():
                        m.weight[m.padding_idx].zero_()
            elif isinstance(m, nn.LayerNorm):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)

    def native_forward(self, input_ids, attention_mask, hooks=None):
        """Returns (pooled, last_hidden) in the compute dtype (autograd-connected)."""
        from .bert import BertEncoderEngine
        from .functions import BertFn
        f = self.native_flat()
        if attention_mask is None:
            attention_mask = torch.ones_like(input_ids)
        eng = BertEncoderEngine(self, f, self.compute_dtype())
        return BertFn.apply(input_ids, attention_mask, self._anchor(input_ids.device), eng, torch.is_grad_enabled(),
                            new_seed(), hooks)

    def forward(self, input_ids=None, attention_mask=None, token_type_ids=None, **kwargs):
        if token_type_ids is not None and bool((token_type_ids != 0).any()):
            raise NotImplementedError("native BertModel supports token_type_ids == 0 (the reference passes none)")
        B, L = input_ids.shape
        pooled, last = self.native_forward(input_ids, attention_mask)
        return BertOutput(last.view(B, L, -1), pooled)
