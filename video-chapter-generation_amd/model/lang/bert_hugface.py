"""Drop-in for reference model/lang/bert_hugface.py:13-132 (BertHugface).

`base_model` is a BERT-base encoder with HF parameter names, executed by libvcg_hip. The
reference's `BertModel.from_pretrained('bert-base-uncased')` needs the network; here the model
is built from the bert-base config (random init, 109,482,240 parameters as bert_hugface.py:31
reports) and a local HF-format state dict can be loaded via `checkpoint=` or $VCG_BERT_CHECKPOINT.
"""
import logging
import os

import torch
import torch.nn as nn

from vcg_hip.nn import BertConfig, BertModel, NativeRoot
from vcg_hip.optim import configure_adamw

logger = logging.getLogger(__name__)


def _load_hf_state(model, path):
    if path.endswith(".safetensors"):
        from safetensors.torch import load_file
        sd = load_file(path)
    else:
        sd = torch.load(path, map_location="cpu", weights_only=True)
        if "model_state_dict" in sd:
            sd = sd["model_state_dict"]
    sd = {k[len("bert."):] if k.startswith("bert.") else k: v for k, v in sd.items()}
    sd = {k: v for k, v in sd.items() if not k.endswith("position_ids") and not k.endswith("token_type_ids")}
    missing, unexpected = model.load_state_dict(sd, strict=False)
    logger.info("loaded %s (missing %d, unexpected %d)", path, len(missing), len(unexpected))


class BertHugface(NativeRoot, nn.Module):
    def __init__(self, pretrain_stage=True, checkpoint=None, config=None):
        super().__init__()
        self.pretrain_stage = pretrain_stage
        config = config if config is not None else BertConfig(output_attentions=True)
        self.base_model = BertModel(config)
        ckpt = checkpoint or os.environ.get("VCG_BERT_CHECKPOINT")
        if ckpt:
            _load_hf_state(self.base_model, ckpt)
        self.vocab_size = self.base_model.config.vocab_size
        self.embed_size = self.base_model.config.hidden_size
        self.head = nn.Linear(self.embed_size, self.vocab_size, bias=False)
        self.head.weight.data.normal_(mean=0.0, std=0.02)
        print("backbone's parameters: ", sum(p.numel() for p in self.base_model.parameters()))

    def build_chapter_head(self):
        self.head = nn.Linear(self.embed_size, 2)

    def fix_backbone(self):
        for pn, p in self.named_parameters():
            if "pooler" in pn or "head" in pn:
                continue
            p.requires_grad = False

    def configure_optimizers(self, train_config):
        return configure_adamw(self, train_config)

    def forward(self, text_ids, attention_mask, get_attention=False):
        from vcg_hip.linear_head import linear_head
        if self.pretrain_stage:
            raise NotImplementedError("MLM pre-training head is outside the video-segment-point path (SURVEY §2 #3b)")
        base_output = self.base_model(input_ids=text_ids, attention_mask=attention_mask)
        return linear_head(self, self.head, base_output.pooler_output)
