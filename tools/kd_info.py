"""Register / LDS / scratch figures of kernels in libvio360.so builds (code-object metadata, CPU only).
usage: python tools/kd_info.py <lib.so> [<lib.so> ...] [--match substr]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import test_build as tb  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
match = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--match=")), "ph_")
for lib in args:
    blob = open(lib, "rb").read()
    print("==", lib)
    for co in tb._gfx950_code_objects(blob):
        for kd in tb._kernel_descriptors(co):
            if match in kd[".name"]:
                print(f"  {kd['.name'][:70]:70s} vgpr={kd['.vgpr_count']:4d} agpr={kd.get('.agpr_count', 0):3d} "
                      f"sgpr={kd['.sgpr_count']:3d} lds={kd['.group_segment_fixed_size']:6d} "
                      f"scratch={kd['.private_segment_fixed_size']:4d} spill_v={kd.get('.vgpr_spill_count', 0)}")
