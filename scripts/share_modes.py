#!/usr/bin/env python3
"""How reproducible one GPU's strong-scaling shares are across fresh processes: runs bench.py's
strong_share child (bench.py --strong-share-child) REPS times under each environment setting and
prints every process's slowest-rank ms per N. Settings: GPU_MAX_HW_QUEUES 8 and 16, and
MFX_SHARE_TORCH_FIRST=1 (torch's stream pools created before the ranks' contexts); `inflight`: 2, 3
or 4 frames in flight; `pool`: each context's stream from a pool the process creates once
(MFX_STREAM_POOL=3) against a stream per context. Usage: share_modes.py [REPS] [inflight|pool]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 3
    settings = [("hwq8", {"GPU_MAX_HW_QUEUES": "8"}), ("hwq16", {"GPU_MAX_HW_QUEUES": "16"}),
                ("hwq8_torch_first", {"GPU_MAX_HW_QUEUES": "8", "MFX_SHARE_TORCH_FIRST": "1"})]
    if len(sys.argv) > 2 and sys.argv[2] == "pool":  # each rank's contexts on streams created once (MFX_STREAM_POOL)
        settings = [("fresh_streams", {"GPU_MAX_HW_QUEUES": "8"}),
                    ("stream_pool3", {"GPU_MAX_HW_QUEUES": "8", "MFX_STREAM_POOL": "3"})]
    if len(sys.argv) > 2 and sys.argv[2] == "inflight":  # frames in flight per small share: 3 (default) vs 4
        settings = [("nif3", {"GPU_MAX_HW_QUEUES": "8"}), ("nif4", {"GPU_MAX_HW_QUEUES": "8", "MFX_FRAMES_IN_FLIGHT": "4"}),
                    ("nif2", {"GPU_MAX_HW_QUEUES": "8", "MFX_FRAMES_IN_FLIGHT": "2"})]
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--strong-share-child", "11400", "30.9"]
    for r in range(reps):  # interleaved: setting after setting, round after round
        for name, env in settings:
            p = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=dict(os.environ, **env))
            if p.returncode != 0:
                print(name, "FAILED", p.stderr[-1500:], flush=True)
                continue
            d = json.loads(p.stdout.strip().splitlines()[-1])
            print(name, r, json.dumps({n: v["slowest_rank_ms"] for n, v in d["shares"].items()}), flush=True)


if __name__ == "__main__":
    main()
