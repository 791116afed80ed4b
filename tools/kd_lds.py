"""Static LDS / registers / scratch of the library's gfx950 kernels whose name contains a pattern.
usage: python tools/kd_lds.py [pattern] [lib]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_build as tb  # noqa: E402

pat = sys.argv[1] if len(sys.argv) > 1 else ""
lib = sys.argv[2] if len(sys.argv) > 2 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                        "360_visual_inertial_odometry_amd", "libvio360.so")
blob = open(lib, "rb").read()
for co in tb._gfx950_code_objects(blob):
    for kd in tb._kernel_descriptors(co):
        if pat in kd[".name"]:
            print(f'{kd[".name"][:90]:90s} lds {kd[".group_segment_fixed_size"]:6d} vgpr {kd[".vgpr_count"]:4d} '
                  f'sgpr {kd[".sgpr_count"]:3d} scratch {kd[".private_segment_fixed_size"]}')
