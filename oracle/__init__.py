"""ORACLE — TEST INFRASTRUCTURE ONLY.

A plain CPU (torch fp32 functional) restatement of the reference's video-segment-point path, used
ONLY by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, and ONLY as the checker /
CPU baseline. The product (video-chapter-generation_amd/) never imports it and has no CPU path.

Pinning: the restatement is checked against golden vectors produced by running the reference's own
modules in this container (tools/oracle/make_golden.py -> tests/golden/*.npz): reference TwoStream /
ChapterHead (model/fusion/two_stream.py), TemporalShift (ops/temporal_shift.py), eval_utils
(eval_utils/eval_utils.py), with transformers' BertModel as lang_model. torchvision is absent, so the
ResNet-50 trunk inside the golden run is our own restatement of torchvision's topology wrapped by the
reference TemporalShift — ResNet arithmetic parity is therefore "parity unpinned" beyond topology
(SURVEY §8c). The index logic (windows, labels, frame gather) is restated from
data/youtube_dataset.py:64-194 and video_chapter_youtube_dataset/flat_video2clip_for_quick_infer.py:64-120.
"""
