"""Drop-in for reference model/vision/resnet50.py:9-73 (plain ResNet-50 image model, no TSM)."""
import torch.nn as nn

from ops.basic_ops import Identity
from vcg_hip.nn import NativeRoot, ResNet50
from vcg_hip.optim import configure_adamw


class Resnet50(NativeRoot, nn.Module):
    def __init__(self, segments_size, pretrain_stage=True):
        super().__init__()
        self.pretrain_stage = pretrain_stage
        self.segments_size = segments_size
        self.base_model = ResNet50()
        self.feature_dim = self.base_model.fc.in_features
        self.base_model.fc = Identity()
        self.head = None

    def build_chapter_head(self):
        self.head = nn.Linear(self.segments_size * self.feature_dim, 2)

    def configure_optimizers(self, train_config):
        return configure_adamw(self, train_config)

    def forward(self, x):
        from vcg_hip.linear_head import linear_head
        batch_size = x.shape[0]
        x = x.reshape(batch_size * x.shape[1], *x.shape[2:])
        out = self.base_model(x)
        out = out.view(batch_size, -1)
        return linear_head(self, self.head, out)
