"""Per-kernel durations from rocprofv3 sqlite output (rocpd `kernels` view), split by grid shape.

    python tools/kstats_db.py <dir-or-db> [name-substring ...]
"""
import glob
import os
import sqlite3
import statistics
import sys


def main():
    path, subs = sys.argv[1], sys.argv[2:]
    dbs = [path] if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)
    d = {}
    for f in dbs:
        c = sqlite3.connect(f)
        for name, dur, gx, gy in c.execute("select name, duration, grid_x, grid_y from kernels"):
            if subs and not any(x in name for x in subs):
                continue
            key = (name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48], gx, gy)
            d.setdefault(key, []).append(dur / 1e3)
    for (n, gx, gy), v in sorted(d.items()):
        print(f"{n:48s} grid {gx:>8}x{gy:<3} n={len(v):4d} med={statistics.median(v):8.2f}us min={min(v):8.2f}us")


if __name__ == "__main__":
    main()
