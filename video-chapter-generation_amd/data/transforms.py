"""The torchvision transforms the reference drivers compose (train_video_segment_point.py:377-386), restated
(torchvision is not a dependency here):

    train: Compose([RandomApply([ColorJitter()], p=0.5), ToTensor(), Normalize(IMAGENET mean, std)])
    test:  Compose([ToTensor(), Normalize(IMAGENET mean, std)])

ColorJitter() with its default arguments (brightness = contrast = saturation = hue = 0) leaves the image
unchanged, so both pipelines are ToTensor + Normalize: PIL RGB u8 [H, W, 3] -> f32 [3, H, W] in [0, 1] -> (x -
mean) / std, per channel, in fp32. The GPU ingest kernel (vcg_window_frames_u8) computes the same map.
"""

import numpy as np
import torch

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)


class Compose:
    def __init__(self, transforms):
        self.transforms = list(transforms)

    def __call__(self, x):
        for t in self.transforms:
            x = t(x)
        return x


class RandomApply:
    def __init__(self, transforms, p=0.5):
        self.transforms, self.p = list(transforms), p

    def __call__(self, x):
        if self.p < torch.rand(1).item():  # torchvision RandomApply draws from torch's RNG
            return x
        for t in self.transforms:
            x = t(x)
        return x


class ColorJitter:
    """Only the default (no-op) jitter the reference uses is supported."""

    def __init__(self, brightness=0, contrast=0, saturation=0, hue=0):
        if any(v not in (0, None) for v in (brightness, contrast, saturation, hue)):
            raise NotImplementedError("ColorJitter with non-zero ranges is not on the reference path")

    def __call__(self, img):
        return img


class ToTensor:
    def __call__(self, img):
        a = np.array(img, dtype=np.uint8)  # a writable copy of the PIL image
        if a.ndim == 2:
            a = a[:, :, None]
        return torch.from_numpy(np.ascontiguousarray(a)).permute(2, 0, 1).float().div(255.0)


class Normalize:
    def __init__(self, mean, std):
        self.mean = torch.tensor(mean, dtype=torch.float32)[:, None, None]
        self.std = torch.tensor(std, dtype=torch.float32)[:, None, None]

    def __call__(self, x):
        return (x - self.mean) / self.std


def train_vision_preprocess():
    return Compose([RandomApply([ColorJitter()], p=0.5), ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)])


def test_vision_preprocess():
    return Compose([ToTensor(), Normalize(IMAGENET_MEAN, IMAGENET_STD)])
