"""End-to-end rate of the reference-side binding: the
binding's hand-off (integration/aqz_handoff.hh) driven by
tests/native/handoff_replay in timing mode on C2 frames (u16 2048^2, 5 levels
with 128-px chunks... the reference rule at 256-px chunks: 4 levels),
camera-like frames made in the replay, every chunk copied out of the pinned
hand-off buffers by a pool of writer threads (GpuArray::write_unit without
the shard I/O).  One JSON line per run.

  python3 tools/binding_e2e.py [--frames 512] [--codecs raw,lz4,...]
  python3 tools/binding_e2e.py --exec ...   the binding itself
      (oracle/_ref/binding_exec: GpuMultiscaleArray / GpuArray over the test
      doubles of Array / MultiscaleArray / Shard, as ZarrStream_s drives it --
      write_frame per frame, the chunk jobs on the reference's ThreadPool,
      finalize; the shard doubles keep sizes only)
"""
import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "tests", "native", "handoff_replay")
EXEC = os.path.join(REPO, "oracle", "_ref", "binding_exec")
CODECS = {"raw": (0, 0, 0), "lz4": (1, 5, 1), "lz4-bit": (1, 5, 2),
          "blosc-zstd": (2, 5, 1), "blosc-zstd-bit": (2, 5, 2), "zstd-1": (3, 1, 0),
          "zstd-3": (3, 3, 0)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=512)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--codecs", default="raw,lz4,lz4-bit,blosc-zstd,zstd-1")
    ap.add_argument("--copy-threads", type=int, default=8)
    ap.add_argument("--pool-threads", type=int, default=16)
    ap.add_argument("--host-slots", type=int, default=3)
    ap.add_argument("--placement-tries", type=int, default=0)
    ap.add_argument("--level0", default="", choices=["", "host", "device"],
                    help="force the level-0 side (default: the binding's choice)")
    ap.add_argument("--exec", action="store_true",
                    help="run the binding itself (binding_exec) instead of the replay")
    args = ap.parse_args()
    env = dict(os.environ)
    if args.level0:
        env["AQZ_REPLAY_LEVEL0"] = args.level0
    dims = [(2, 0, 64, 1), (0, 2048, 256, 1), (0, 2048, 256, 1)]
    for name in args.codecs.split(","):
        with tempfile.TemporaryDirectory() as d:
            job = os.path.join(d, "job.bin")
            with open(job, "wb") as f:
                f.write(b"AQZ2" + struct.pack("<I", len(dims)))
                for x in dims:
                    f.write(struct.pack("<iIII", *x))
                f.write(struct.pack("<iiIIiiiiIIIIIQQ", 1, 1, args.batch, args.host_slots, 0,
                                    *CODECS[name], args.copy_threads, args.pool_threads, 1,
                                    args.placement_tries, 1, args.frames, 2048 * 2048 * 2))
            r = subprocess.run([EXEC if args.exec else EXE, job, "-"], capture_output=True, text=True, timeout=600,
                               env=env)
            if r.returncode != 0:
                sys.exit(r.stdout[-2000:] + r.stderr[-2000:])
            s = json.loads(r.stdout.strip().splitlines()[-1])
            s["codec_name"] = name
            s["harness"] = "binding_exec" if args.exec else "handoff_replay"
            s["workload"] = ("C2 frames u16 2048x2048, 256x256 chunks (t-chunk 64), 4 levels "
                             "(reference rule), camera-like, pageable frame per write_frame "
                             "-> binding hand-off -> sink pool copy")
            print(json.dumps(s), flush=True)


if __name__ == "__main__":
    main()
