"""Generate tests/golden/windows.json: pins for the window / label / frame-index logic (row a10).

Runs only in the build container. It imports the REFERENCE's `data/common_utils.py` by path (pandas,
re and pickle only, so it imports here) and records `extract_first_timestamp` on a list of chapter
timestamp strings. The windowing lines themselves are in modules that cannot be imported here
(torchvision / youtube_transcript_api are absent). For those, the file also holds known answers
worked out by hand from `youtube_dataset.py:89-114` and `flat_video2clip_for_quick_infer.py:62-106`.
The test suite checks these answers against both `oracle/windows.py` and `data/clip_windows.py`.
Usage: python tools/oracle/make_golden_data.py
"""
import importlib.util
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/video_chapter_generation"

TIMESTAMPS = [
    "00:00 Intro", "0:45 setup", "01:02:03 deep dive 0:45", "1:02:03 part two", "12:34 - the end",
    "no timestamp here", "Chapter 3 (3:07)", "10:00:00 marathon", "5:5 bad", "07:59 x 07:58 y",
    "[4:03] bracketed", "2:00:00 and 59:59", "001:30 three digits", "0:04 edge", "0:03 too early",
]


def main():
    spec = importlib.util.spec_from_file_location("ref_common_utils", os.path.join(REF, "data", "common_utils.py"))
    cu = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(cu)
    ts = [{"s": s, "sec": cu.extract_first_timestamp(s)[0], "desc": cu.extract_first_timestamp(s)[1]}
          for s in TIMESTAMPS]

    # Hand-derived known answers (T = 16, max_offset = 2: threshold 14/18 = 0.777…).
    # Video of 40 frames: windows start at 0, 4, ..., 20 (range(0, 24, 4)).
    # Cut point 20: window [12,28) vs [12,28) -> IoU 1; [8,24) -> (24-12)/(28-8) = 0.6;
    # [16,32) -> (28-16)/(32-12) = 0.6. Only s = 12 is positive.
    # Cut point 10 (eval filter keeps 4 <= cp <= 36): [0,16) vs [2,18) -> 14/18 = 0.777… >= thr -> 1;
    # [4,20) vs [2,18) -> 14/18 -> 1.
    known = {
        "video40": {
            "image_num": 40, "T": 16, "cut_points": [10, 20],
            "windows": [[0, 16], [4, 20], [8, 24], [12, 28], [16, 32], [20, 36]],
            "labels": [1, 1, 0, 1, 0, 0],
            # frame numbers: s <= 2 or s >= 40 - 16 - 2 = 22 -> +1, else +3
            "frames_s0": list(range(1, 17)), "frames_s4": list(range(7, 23)), "frames_s20": list(range(23, 39)),
        },
        # subtitles with start strictly inside (s - 1, e + 1); an empty first text adds no separator
        "subtitles": {
            "subs": [{"start": 3.0, "text": "too early"}, {"start": 3.5, "text": ""}, {"start": 4.0, "text": "a"},
                     {"start": 19.9, "text": "b"}, {"start": 21.0, "text": "late"}],
            "window": [4, 20], "text": "a b",
        },
        # train keeps cp <= image_num, eval keeps cp <= image_num - 4
        "filters": {"image_num": 40, "secs": [3, 4, 36, 37, 40, 41, -1],
                    "train": [4, 36, 37, 40], "eval": [4, 36]},
    }
    out = {"extract_first_timestamp": ts, "known": known,
           "source": "reference data/common_utils.py (imported) + hand-derived answers"}
    path = os.path.join(REPO, "tests", "golden", "windows.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
