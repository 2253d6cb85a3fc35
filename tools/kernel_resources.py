"""Per-kernel resource usage (scratch, VGPR/AGPR, LDS, SGPR) of the built gfx950 code objects.

Reads the ``.hip_fatbin`` section of the in-tree extension, splits it into its clang offload
bundles (one per translation unit), extracts each gfx950 code object and prints the AMDHSA
kernel metadata.  Used by ``tests/test_kernel_resources.py`` to keep every hot kernel free of
scratch spills (a spill inside a k-loop costs a global-memory round trip per use).

    python tools/kernel_resources.py [path/to/_C*.so]
"""
from __future__ import annotations

import glob
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def default_so() -> str:
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    hits = sorted(glob.glob(os.path.join(here, "pytorch_distributed_mnist_amd", "_C*.so")))
    if not hits:
        raise FileNotFoundError("extension not built (python -m pytorch_distributed_mnist_amd.build)")
    return hits[0]


def code_objects(so: str) -> list[bytes]:
    """gfx950 code objects of every offload bundle in the library's .hip_fatbin section."""
    with tempfile.TemporaryDirectory() as td:
        sec = os.path.join(td, "fatbin")
        subprocess.run([os.path.join(LLVM, "llvm-objcopy"), f"--dump-section=.hip_fatbin={sec}",
                        so, os.path.join(td, "discard")], check=True, capture_output=True)
        data = open(sec, "rb").read()
    out = []
    pos = data.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", data, pos + len(MAGIC))
        p = pos + len(MAGIC) + 8
        for _ in range(n):
            off, size, tl = struct.unpack_from("<QQQ", data, p)
            triple = data[p + 24:p + 24 + tl].decode()
            p += 24 + tl
            if "gfx950" in triple and size:
                out.append(data[pos + off:pos + off + size])
        pos = data.find(MAGIC, p)
    return out


_FIELDS = ("private_segment_fixed_size", "group_segment_fixed_size", "vgpr_count", "agpr_count",
           "sgpr_count", "vgpr_spill_count", "sgpr_spill_count")


def kernels(so: str | None = None) -> dict[str, dict[str, int]]:
    """{kernel symbol: metadata fields} over all code objects of the extension."""
    res: dict[str, dict[str, int]] = {}
    with tempfile.TemporaryDirectory() as td:
        for i, co in enumerate(code_objects(so or default_so())):
            path = os.path.join(td, f"co{i}.elf")
            open(path, "wb").write(co)
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", path],
                                   check=True, capture_output=True, text=True).stdout
            # kernel entries are the two-space-indented list items of amdhsa.kernels
            blocks = re.split(r"\n  - ", notes)
            for b in blocks:
                m = re.search(r"\.name:\s+(\S+)", b)
                if not m or ".kd" in m.group(1):
                    continue
                f = {}
                for k in _FIELDS:
                    mm = re.search(rf"(?:^|\n)\s*\.{k}:\s+(\d+)", b)
                    if mm:
                        f[k] = int(mm.group(1))
                if "vgpr_count" in f:
                    res[m.group(1)] = f
    return res


def main(argv):
    so = argv[0] if argv else None
    ks = kernels(so)
    print(f"{'kernel':58s} {'scratch':>7s} {'vgpr':>5s} {'agpr':>5s} {'sgpr':>5s} {'lds':>7s}")
    for name, f in sorted(ks.items()):
        short = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", name)[:58]
        print(f"{short:58s} {f.get('private_segment_fixed_size', -1):7d} {f.get('vgpr_count', -1):5d} "
              f"{f.get('agpr_count', -1):5d} {f.get('sgpr_count', -1):5d} "
              f"{f.get('group_segment_fixed_size', -1):7d}")


if __name__ == "__main__":
    main(sys.argv[1:])
