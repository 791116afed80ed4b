"""Build hygiene (CPU): header dependencies are generated, so a header change rebuilds every object
that includes it, and the library's translation units agree on the cross-TU struct layouts.

A stale ba_kernel.o after a GbaArgs change once faulted the global VIBA path on the GPU; these tests
pin the two guards against that class of fault (csrc/Makefile -MMD -MP, ba_types.h / ba_global.h
static_asserts + vio_layout_check)."""
import os
import re
import struct
import subprocess


import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "360_visual_inertial_odometry_amd", "csrc")


def _make(*args):
    return subprocess.run(["make", "-C", CSRC, "ARCH=gfx950", *args], capture_output=True, text=True)


def _includers(header):
    """translation units whose generated .d file lists `header`"""
    out = []
    for d in sorted(os.listdir(os.path.join(CSRC, "build"))):
        if d.endswith(".d") and re.search(r"(^|[\s/])" + re.escape(header) + r"\b",
                                          open(os.path.join(CSRC, "build", d)).read()):
            out.append(d[:-2])
    return out


@pytest.fixture(scope="module")
def built(vio):
    vio.lib()  # the library exists (build() ran)
    if not os.path.isdir(os.path.join(CSRC, "build")):
        pytest.skip("objects not built in-tree")
    if _make("-q").returncode != 0:
        pytest.skip("library not up to date with its sources (run the build first)")


@pytest.mark.parametrize("header,must", [
    ("ba_types.h", {"ba_kernel", "ba_host", "ba_global_host"}),
    ("ba_global.h", {"ba_kernel", "ba_global", "ba_global_host"}),
    ("chol_dev.h", {"ba_kernel", "ba_global"}),
    ("vio360.h", {"ba_kernel", "ba_host", "ba_global", "ba_global_host", "tracker_host"}),
])
def test_touching_a_header_rebuilds_its_dependents(built, header, must):
    deps = set(_includers(header))
    assert must <= deps, (header, sorted(deps))
    # `make -q -W h` = "is anything out of date if h were touched" (no file is modified)
    path = "../../include/" + header if header == "vio360.h" else header  # as the .d files name it
    assert _make("-q", "-W", path).returncode != 0
    dry = _make("-n", "-W", path).stdout
    rebuilt = set(re.findall(r"-o build/(\w+)\.o", dry))
    assert rebuilt == deps, (header, sorted(rebuilt), sorted(deps))


def test_translation_units_agree_on_struct_layouts(vio):
    assert vio.lib().vio_layout_check() == 0


# ---- code-object metadata of the shipped library (no GPU needed) ----
_BUNDLE = b"__CLANG_OFFLOAD_BUNDLE__"


def _gfx950_code_objects(blob):
    """the gfx950 ELF code objects of every (uncompressed) clang offload bundle in the library"""
    i = 0
    while True:
        i = blob.find(_BUNDLE, i)
        if i < 0:
            return
        n, = struct.unpack_from("<Q", blob, i + 24)
        p = i + 32
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", blob, p)
            p += 24
            triple = blob[p:p + tl].decode()
            p += tl
            if "gfx950" in triple:
                yield blob[i + off:i + off + size]
        i += len(_BUNDLE)



def _msgpack():
    """msgpack (the code-object metadata format) -- only the code-object tests need it: skipped without it"""
    return pytest.importorskip("msgpack")

def _kernel_descriptors(co):
    """amdhsa.kernels entries of a code object's NT_AMDGPU_METADATA note (msgpack)"""
    shoff, = struct.unpack_from("<Q", co, 0x28)
    shentsize, shnum = struct.unpack_from("<HH", co, 0x3A)
    for k in range(shnum):
        sh = shoff + k * shentsize
        typ, = struct.unpack_from("<I", co, sh + 4)
        off, size = struct.unpack_from("<QQ", co, sh + 0x18)
        if typ != 7:  # SHT_NOTE
            continue
        p = off
        while p < off + size:
            nsz, dsz, nt = struct.unpack_from("<III", co, p)
            p += 12
            name = co[p:p + nsz]
            p += (nsz + 3) & ~3
            desc = co[p:p + dsz]
            p += (dsz + 3) & ~3
            if nt == 32 and name.startswith(b"AMDGPU"):
                yield from _msgpack().unpackb(desc, raw=False)["amdhsa.kernels"]


def test_cluster_kernel_has_no_scratch(vio):
    """ph_cluster_kernel (the single-window route's persistent launch) keeps every value in registers or LDS:
    its private segment is zero bytes (no spills, no call stack) and it stays within one workgroup per CU's
    register file (512 VGPRs incl. AGPRs)"""
    blob = open(vio.lib()._name, "rb").read()
    found = [kd for co in _gfx950_code_objects(blob) for kd in _kernel_descriptors(co)
             if "ph_cluster_kernel" in kd[".name"]]
    assert len(found) == 1, [kd[".name"] for kd in found]
    kd = found[0]
    assert kd[".private_segment_fixed_size"] == 0, kd[".private_segment_fixed_size"]
    assert kd[".vgpr_count"] <= 512  # the unified file: arch VGPRs + AGPRs


def test_wide_phase_kernels_have_no_scratch(vio):
    """the phase route's per-window kernels that run one workgroup per window across the chip (ph_prep,
    ph_back, ph_solve) touch no scratch: a workgroup's first private-segment access cost ph_prep ≈ 25 k
    cycles per window at 256 windows (profiles/r5s_*).  (The global solver's one-workgroup diagonal
    launches keep their call and its 12-B stack: inlined they were 5 % slower, profiles/r5s_gba_inline_ab.log.)"""
    blob = open(vio.lib()._name, "rb").read()
    want = ("ph_prep_kernel", "ph_back_kernel", "ph_back_x_kernel", "ph_solve_kernel")
    found = {}
    for co in _gfx950_code_objects(blob):
        for kd in _kernel_descriptors(co):
            for w in want:
                if w + "E" in kd[".name"]:
                    found[w] = kd[".private_segment_fixed_size"]
    assert set(found) == set(want), found
    assert all(v == 0 for v in found.values()), found


def test_walk_kernel_fits_five_waves_per_simd(vio):
    """ph_back_kernel (the 256-window step's largest kernel) stays at <= 96 VGPRs, i.e. five waves per SIMD with
    its 28.3 KB of LDS (five workgroups per CU): at 110 VGPRs / four waves it took 107 us per launch against
    98 us (profiles/r6g_ab_back.log)"""
    blob = open(vio.lib()._name, "rb").read()
    found = [kd for co in _gfx950_code_objects(blob) for kd in _kernel_descriptors(co)
             if "ph_back_kernelE" in kd[".name"]]
    assert len(found) == 1, [kd[".name"] for kd in found]
    assert found[0][".vgpr_count"] <= 96, found[0][".vgpr_count"]
    assert found[0][".group_segment_fixed_size"] * 5 <= 160 * 1024, found[0][".group_segment_fixed_size"]
