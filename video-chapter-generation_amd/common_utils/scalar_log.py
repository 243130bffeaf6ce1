"""Scalar logging for the drivers: the reference writes tensorboard scalars through SummaryWriter
(`train_video_segment_point.py:315-316,244-248,279-281`). tensorboard is not installed in this image, so
`summary_writer` falls back to a writer with the same `add_scalar(tag, value, step)` call that appends one JSON
line per scalar to <log_dir>/scalars.jsonl."""
import json
import os


class JsonlSummaryWriter:
    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "scalars.jsonl")
        self._f = open(self.path, "a")

    def add_scalar(self, tag, value, step):
        self._f.write(json.dumps({"tag": tag, "value": float(value), "step": int(step)}) + "\n")
        self._f.flush()

    def close(self):
        self._f.close()


def summary_writer(log_dir):
    try:
        from torch.utils.tensorboard import SummaryWriter
        return SummaryWriter(log_dir)
    except ImportError:
        return JsonlSummaryWriter(log_dir)
