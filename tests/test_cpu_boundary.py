"""Drop-in boundary: TwoStream accepts the encoders the REFERENCE builds -- a transformers BertModel
(bert_hugface.py:20) and a torchvision-topology resnet50 with TemporalShift around every bottleneck conv1 and
fc = Identity (resnet50_tsm.py:10-20) -- and converts them to the native modules with identical weights, buffers
and shift geometry (no compute: CPU)."""
import os
import sys

import pytest
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tools", "oracle"))


def _foreign_encoders(T):
    from transformers import BertConfig, BertModel
    import tv_resnet
    from ops.temporal_shift import TemporalShift
    cfg = BertConfig(vocab_size=100, hidden_size=64, num_hidden_layers=2, num_attention_heads=4,
                     intermediate_size=128, hidden_dropout_prob=0.05, attention_probs_dropout_prob=0.02)
    torch.manual_seed(0)
    lang = BertModel(cfg, add_pooling_layer=True)
    vis = tv_resnet.ResNet()
    for layer in (vis.layer1, vis.layer2, vis.layer3, vis.layer4):  # the reference's blockres placement
        for b in layer:
            b.conv1 = TemporalShift(b.conv1, n_segment=T, n_div=8)
    vis.fc = torch.nn.Identity()
    with torch.no_grad():  # non-default BN buffers so the copy is visible
        for m in vis.modules():
            if isinstance(m, torch.nn.BatchNorm2d):
                m.running_mean.uniform_(-1, 1)
                m.running_var.uniform_(0.5, 2)
    return lang, vis


def test_two_stream_adopts_reference_encoders():
    from model.fusion import two_stream
    from vcg_hip.nn import BertModel, ResNet50
    T = 4
    lang, vis = _foreign_encoders(T)
    m = two_stream.TwoStream(lang, vis, 64, 2048, T, 128)
    assert isinstance(m.lang_model, BertModel) and isinstance(m.vision_model, ResNet50)
    c = m.lang_model.config
    assert (c.hidden_size, c.num_hidden_layers, c.num_attention_heads, c.intermediate_size) == (64, 2, 4, 128)
    assert (c.hidden_dropout_prob, c.attention_probs_dropout_prob) == (0.05, 0.02)
    for name, ref in ((n, t) for n, t in lang.state_dict().items() if not n.endswith(("position_ids", "token_type_ids"))):
        assert torch.equal(m.lang_model.state_dict()[name], ref), name
    nsd = m.vision_model.state_dict()
    assert set(nsd) == set(vis.state_dict())
    for name, ref in vis.state_dict().items():
        assert torch.equal(nsd[name], ref), name
    shifts = [x for x in m.vision_model.modules() if type(x).__name__ == "TemporalShift"]
    assert len(shifts) == 16 and all(s.n_segment == T and s.fold_div == 8 for s in shifts)
    # the native modules are used as given
    m2 = two_stream.TwoStream(m.lang_model, m.vision_model, 64, 2048, T, 128)
    assert m2.lang_model is m.lang_model and m2.vision_model is m.vision_model


def test_two_stream_rejects_other_encoders():
    from model.fusion import two_stream
    with pytest.raises(TypeError):
        two_stream.TwoStream(torch.nn.Linear(2, 2), torch.nn.Linear(2, 2), 768, 2048, 4, 128)
