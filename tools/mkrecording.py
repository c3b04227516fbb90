"""Write a synthetic recording in the reference's offline layout (aicp_input_poses.csv +
cloud_<c>_<s>_<ns>.pcd, binary PCD as app_ros.cpp:155-172 writes them) for `bench.py --data`.

usage: python tools/mkrecording.py OUT_DIR [n_clouds] [n_points]
Cloud 0 is a reference-like scan and clouds 1.. are the C2 sequence's readings; poses carry the
sensor origins (identity rotation)."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aicp_mapping_amd import cloud_io as io  # noqa: E402
from aicp_mapping_amd import synthetic as sy  # noqa: E402


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 21
    pts = int(sys.argv[3]) if len(sys.argv) > 3 else 120000
    os.makedirs(out, exist_ok=True)
    seq = sy.make_sequence(n - 1, n, pts, seed=1)
    clouds = [seq[0].ref] + [p.read for p in seq]
    origins = [seq[0].ref_origin] + [p.read_origin for p in seq]
    recs = []
    for i, (P, o) in enumerate(zip(clouds, origins)):
        T = np.eye(4)
        T[:3, 3] = o
        u = 1500000000000000 + i * 100000
        sec = u // 1000000
        rec = io.IsometryWithTime(T, sec, u - sec * 1000000, i)
        io.save_pcd_xyz(io.cloud_file_name(out, i, rec.sec, rec.nsec), P)
        recs.append(rec)
    io.write_pose_file(os.path.join(out, "aicp_input_poses.csv"), recs)
    print("wrote %d clouds to %s" % (n, out))


if __name__ == "__main__":
    main()
