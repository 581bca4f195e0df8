"""Copy one gpu_session.sh run's results into profiles/ under a round prefix.

    python tools/collect_session.py TAG            # gpurun_out/TAG/... -> profiles/TAG_...

Bench lines (``*.json`` whose last line is a JSON object) keep their name; every rocprofv3
``*_kernel_stats.csv`` under the session becomes ``TAG_<dir>_kernel_stats.csv``; stamps and
pytest / smoke logs are copied as they are.  gpurun_out/ is scratch; profiles/ is what the
judge reads.
"""
import glob
import json
import os
import shutil
import sys

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")


def main(tag: str) -> None:
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles")
    done = []
    for path in sorted(glob.glob(os.path.join(src, "**", "*"), recursive=True)):
        if os.path.isdir(path):
            continue
        rel = os.path.relpath(path, src)
        name = None
        if path.endswith(".json"):
            try:
                with open(path) as f:
                    lines = [ln for ln in f.read().splitlines() if ln.strip()]
                json.loads(lines[-1] if lines[-1].startswith("{") else "\n".join(lines))
            except (ValueError, IndexError):
                continue
            name = rel.replace(os.sep, "_")
        elif path.endswith("_kernel_stats.csv"):
            name = os.path.dirname(rel).replace(os.sep, "_") + "_kernel_stats.csv"
        elif path.endswith((".log", ".jsonl")):
            name = rel.replace(os.sep, "_")
        if name:
            out = os.path.join(dst, f"{tag}_{name}")
            shutil.copyfile(path, out)
            done.append(os.path.relpath(out, ROOT))
    print("\n".join(done))


if __name__ == "__main__":
    main(sys.argv[1])
