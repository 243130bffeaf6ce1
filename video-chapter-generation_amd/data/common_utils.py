"""Drop-in for reference data/common_utils.py (the parts on the clip-scorer path).

- `parse_csv_to_list(csv_file)` -- `common_utils.py:6-15`: the dataset CSV (columns videoId, title, duration,
  timestamp) -> (vids, titles, durations, timestamps), each video's timestamp cell split on the "%^&*" delimiter;
- `extract_timestamp`, `extract_first_timestamp` -- `common_utils.py:37-83` (restated in data/clip_windows.py).
"""
import pandas as pd

from .clip_windows import extract_first_timestamp, extract_timestamp  # noqa: F401

TIMESTAMP_DELIMITER = "%^&*"


def parse_csv_to_list(csv_file):
    data = pd.read_csv(csv_file)
    vids = list(data["videoId"].values)
    titles = list(data["title"].values)
    durations = list(data["duration"].values)
    timestamps = [str(x).split(TIMESTAMP_DELIMITER) for x in data["timestamp"].values]
    return vids, titles, durations, timestamps


def write_csv(csv_file, vids, titles, durations, timestamps):
    """The inverse (test fixtures / synthetic corpora written to disk in the reference's format)."""
    pd.DataFrame({"videoId": vids, "title": titles, "duration": durations,
                  "timestamp": [TIMESTAMP_DELIMITER.join(t) for t in timestamps]}).to_csv(csv_file, index=False)
