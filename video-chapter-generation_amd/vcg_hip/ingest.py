"""Clip-batch ingest for the drivers: decoded u8 frames go to the GPU as bytes (a quarter of
the f32 upload the reference makes, `train_video_segment_point.py:149`) and are normalised there, as
ToTensor + Normalize (`train_video_segment_point.py:383-386`), straight into the stem's NHWC layout by
vcg_window_frames_u8 (frame b*T + t: the `(b t)` order of `two_stream.py:183`)."""
import torch

from . import ops


def stage_clips_u8(img_u8, device, dtype):
    """img_u8: [B, T, H, W, 3] uint8 (host or device) -> the stem's input [B*T, H, W, cpad] on `device`."""
    if img_u8.dtype != torch.uint8 or img_u8.dim() != 5 or img_u8.shape[-1] != 3:
        raise ValueError(f"expected uint8 [B,T,H,W,3] clips, got {img_u8.dtype} {tuple(img_u8.shape)}")
    B, T, H, W, _ = img_u8.shape
    frames = img_u8.reshape(B * T, H, W, 3).to(device, non_blocking=True).contiguous()
    idx = torch.arange(B * T, dtype=torch.int64, device=device)
    return ops.window_frames_u8(frames, idx, dtype, cpad=ops.stem_cpad(dtype))


def is_u8_clips(img_clip):
    return torch.is_tensor(img_clip) and img_clip.dtype == torch.uint8 and img_clip.dim() == 5
