"""Drop-in for reference model/vision/resnet50_tsm.py:10-77 (Resnet50TSM).

`base_model` is a torchvision-topology ResNet-50 with TemporalShift on every bottleneck conv1 and
fc = Identity, executed by libvcg_hip. `pretrained=True` ImageNet weights cannot be fetched
offline: weights are torchvision-initialised unless `checkpoint` (a torchvision resnet50 state
dict file) is given.
"""
import torch
import torch.nn as nn

from ops.basic_ops import Identity
from ops.temporal_shift import make_temporal_shift
from vcg_hip.nn import NativeRoot, ResNet50
from vcg_hip.optim import configure_adamw


class Resnet50TSM(NativeRoot, nn.Module):
    def __init__(self, segments_size=8, shift_div=8, pretrain_stage=True, checkpoint=None):
        super().__init__()
        self.pretrain_stage = pretrain_stage
        self.base_model = ResNet50()
        if checkpoint is not None:
            sd = torch.load(checkpoint, map_location="cpu", weights_only=True)
            self.base_model.load_state_dict(sd)
        make_temporal_shift(self.base_model, n_segment=segments_size, n_div=shift_div)
        self.segments_size = segments_size
        self.feature_dim = self.base_model.fc.in_features
        self.base_model.fc = Identity()  # discard last fc layer
        self.head = None

    def build_chapter_head(self):
        self.head = nn.Linear(self.segments_size * self.feature_dim, 2)

    def configure_optimizers(self, train_config):
        return configure_adamw(self, train_config)

    def forward(self, x):
        """x: [B, T, 3, H, W] -> (logits [B, 2], prob [B, 2]) (image-only mode)."""
        from vcg_hip.linear_head import linear_head
        batch_size = x.shape[0]
        x = x.reshape(batch_size * x.shape[1], *x.shape[2:])  # 'b t c h w -> (b t) c h w'
        out = self.base_model(x)
        out = out.view(batch_size, -1)  # concatenate all vision embeddings along the segment dim
        return linear_head(self, self.head, out)
