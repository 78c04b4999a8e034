"""Repeat one binding_exec run (C2 frames, zstd-1 through the hook, 8 pool
threads: the case one AddressSanitizer pass stalled in) N times, each under
its own time limit, with the harness's progress file; one JSON line a run.

  python3 tools/binding_stress.py [--runs 20] [--exe oracle/_ref/binding_exec]
"""
import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=20)
    ap.add_argument("--exe", default=os.path.join(REPO, "oracle", "_ref", "binding_exec"))
    ap.add_argument("--prefix", default="")
    ap.add_argument("--limit", type=int, default=90)
    args = ap.parse_args()
    from oracle_bindings import U16, MEAN, TIME, SPACE, synthetic_frames
    dims = [(TIME, 0, 16, 2), (SPACE, 2048, 256, 1), (SPACE, 2048, 256, 1)]
    frames = synthetic_frames(U16, 5 * 16 + 7, 2048, 2048, 2) & 0x0fff
    frames[20:23] = 0
    prog = os.path.join(REPO, "gpurun_out", "binding_stress_progress.txt")
    os.makedirs(os.path.dirname(prog), exist_ok=True)
    with tempfile.TemporaryDirectory() as d:
        job = os.path.join(d, "job.bin")
        with open(job, "wb") as f:
            f.write(b"AQZ2" + struct.pack("<I", len(dims)))
            for x in dims:
                f.write(struct.pack("<iIII", *x))
            f.write(struct.pack("<iiIIiiiiIIIIIQQ", U16, MEAN, 0, 0, 0, 3, 1, 0, 0, 8, 0, 0, 1,
                                len(frames), frames[0].nbytes))
            f.write(frames.tobytes())
        env = dict(os.environ, BINDING_EXEC_PROGRESS=prog)
        for i in range(args.runs):
            t0 = time.time()
            try:
                r = subprocess.run(args.prefix.split() + [args.exe, job, os.path.join(d, "o")],
                                   capture_output=True, text=True, timeout=args.limit, env=env)
                rc, tail = r.returncode, (r.stdout + r.stderr)[-300:]
            except subprocess.TimeoutExpired:
                rc, tail = "timeout", ""
            print(json.dumps({"run": i, "rc": rc, "seconds": round(time.time() - t0, 2),
                              "tail": tail if rc != 0 else ""}), flush=True)
            if rc != 0:
                sys.exit(1)


if __name__ == "__main__":
    main()
