"""Run bench.py with class attributes set first (same-box A/B of the switches that are class attributes, INTEGRATION.md
§5). usage: python tools/bench_attr.py vcg_hip.bert.BertEncoderEngine.unpad=0 [more=...] -- <bench.py args>"""
import importlib
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "video-chapter-generation_amd"))
cut = sys.argv.index("--") if "--" in sys.argv else len(sys.argv)
sets, rest = sys.argv[1:cut], sys.argv[cut + 1:]
for a in sets:
    path, val = a.split("=", 1)
    mod, cls, attr = path.rsplit(".", 2)
    v = {"0": False, "1": True}.get(val)
    if v is None:
        v = int(val) if val.lstrip("-").isdigit() else val
    setattr(getattr(importlib.import_module(mod), cls), attr, v)
sys.argv = ["bench.py"] + rest
import bench  # noqa: E402

bench.main()
