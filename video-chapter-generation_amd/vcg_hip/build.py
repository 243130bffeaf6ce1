"""Model construction exactly as the reference drivers do it
(train_video_segment_point.py:323-363, test_video_segment_point.py:69-100):

    lang_model = BertHugface(pretrain_stage=False)
    vision_model = Resnet50TSM(segments_size=clip_frame_num, shift_div=8, pretrain_stage=False)
    model = TwoStream(lang_model.base_model, vision_model.base_model, lang_model.embed_size,
                      vision_model.feature_dim, clip_frame_num, hidden_size=128)
    model.build_chapter_head(output_size=2, head_type=head_type)
"""
import contextlib
import io

from . import synth


def build_two_stream(clip_frame_num=16, hidden_size=128, head_type="mlp", dropout=None, seed=None, device=None,
                     precision="fp32", bn_stats=None):
    from model.fusion.two_stream import TwoStream
    from model.lang.bert_hugface import BertHugface
    from model.vision.resnet50_tsm import Resnet50TSM
    from vcg_hip.nn import BertConfig

    cfg = BertConfig(output_attentions=True)
    if dropout is not None:
        cfg.hidden_dropout_prob = dropout
        cfg.attention_probs_dropout_prob = dropout
    with contextlib.redirect_stdout(io.StringIO()):
        lang_model = BertHugface(pretrain_stage=False, config=cfg)
    vision_model = Resnet50TSM(segments_size=clip_frame_num, shift_div=8, pretrain_stage=False)
    model = TwoStream(lang_model.base_model, vision_model.base_model, lang_model.embed_size, vision_model.feature_dim,
                      clip_frame_num, hidden_size)
    model.build_chapter_head(output_size=2, head_type=head_type)
    if dropout is not None and head_type == "attn":
        model.fusion_head.head.attn_drop.p = dropout
    if device is not None:
        model = model.to(device)
    if seed is not None:
        synth.init_params(model, seed)  # on the GPU this runs the HIP generator (bit-identical to numpy)
    if bn_stats is not None:
        synth.load_bn_stats(model, bn_stats)
    model.precision = precision
    return model


def build_model(data_mode="all", clip_frame_num=16, hidden_size=128, head_type="mlp", model_type="r50tsm", seed=None,
                device=None, precision="bf16", dropout=None):
    """The driver's model by `--data_mode` (`train_video_segment_point.py:330-363`): "text" ->
    BertHugface + head, "image" -> Resnet50TSM (or Resnet50) + head, "all" -> TwoStream."""
    if data_mode == "all":
        return build_two_stream(clip_frame_num, hidden_size, head_type, dropout, seed, device, precision)
    if data_mode == "text":
        from model.lang.bert_hugface import BertHugface
        from vcg_hip.nn import BertConfig
        cfg = BertConfig(output_attentions=True)
        if dropout is not None:
            cfg.hidden_dropout_prob = cfg.attention_probs_dropout_prob = dropout
        with contextlib.redirect_stdout(io.StringIO()):
            model = BertHugface(pretrain_stage=False, config=cfg)
    elif data_mode == "image":
        if model_type == "r50tsm":
            from model.vision.resnet50_tsm import Resnet50TSM
            model = Resnet50TSM(segments_size=clip_frame_num, shift_div=8, pretrain_stage=False)
        elif model_type == "r50":
            from model.vision.resnet50 import Resnet50
            model = Resnet50(segments_size=clip_frame_num, pretrain_stage=False)
        else:
            raise RuntimeError(f"Unknown model_type {model_type}")
    else:
        raise RuntimeError(f"Unknown data mode {data_mode}")
    model.build_chapter_head()
    if device is not None:
        model = model.to(device)
    if seed is not None:
        synth.init_params(model, seed)
    model.precision = precision
    return model


def build_window_two_stream(clip_frame_num=16, window_size=1, hidden_size=128, head_type="cross_attn", seed=None,
                            device=None, precision="fp32", bn_stats=None):
    """The window model as the reference DDP driver builds it (train_video_segment_ddp.py:463-486):
    two_stream_window.TwoStream(lang.base_model, vision.base_model, 768, 2048, T, 128, window_size) +
    build_chapter_head(2, head_type)."""
    from model.fusion.two_stream_window import TwoStream
    from model.lang.bert_hugface import BertHugface
    from model.vision.resnet50_tsm import Resnet50TSM
    from vcg_hip.nn import BertConfig

    with contextlib.redirect_stdout(io.StringIO()):
        lang_model = BertHugface(pretrain_stage=False, config=BertConfig(output_attentions=True))
    vision_model = Resnet50TSM(segments_size=clip_frame_num, shift_div=8, pretrain_stage=False)
    model = TwoStream(lang_model.base_model, vision_model.base_model, lang_model.embed_size, vision_model.feature_dim,
                      clip_frame_num, hidden_size, window_size)
    with contextlib.redirect_stdout(io.StringIO()):
        model.build_chapter_head(output_size=2, head_type=head_type)
    if device is not None:
        model = model.to(device)
    if seed is not None:
        synth.init_params(model, seed)
    if bn_stats is not None:
        synth.load_bn_stats(model, bn_stats)
    model.precision = precision
    return model
