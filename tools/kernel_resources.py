"""Development: VGPR / spill / LDS figures of the kernels in the gfx950 code
object of a built libkhmer_hip.so (llvm-readelf notes), filtered by name."""
import re
import subprocess
import sys
import tempfile

so = sys.argv[1]
pat = re.compile(sys.argv[2] if len(sys.argv) > 2 else ".")
LLVM = "/opt/rocm/lib/llvm/bin/"
sec = subprocess.check_output([LLVM + "llvm-readelf", "-S", "-W", so]).decode()
for line in sec.splitlines():
    if ".hip_fatbin" in line:
        parts = line.split()
        i = parts.index(".hip_fatbin")
        off, size = int(parts[i + 3], 16), int(parts[i + 4], 16)
with tempfile.TemporaryDirectory() as d:
    with open(so, "rb") as fh:
        fh.seek(off)
        open(d + "/fb", "wb").write(fh.read(size))
    subprocess.check_call([LLVM + "clang-offload-bundler", "--unbundle", "--type=o", "--input=" + d + "/fb",
                           "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", "--output=" + d + "/co"])
    notes = subprocess.check_output([LLVM + "llvm-readelf", "--notes", d + "/co"]).decode()
for blk in notes.split("- .agpr_count")[1:]:
    m = re.search(r"\.name:\s+(\S+)", blk)
    if not m or not pat.search(m.group(1)):
        continue
    g = lambda k: re.search(r"\." + k + r":\s+(\d+)", blk).group(1)
    print("%-90s vgpr %3s spill %3s sgpr %3s" % (m.group(1)[:90], g("vgpr_count"), g("vgpr_spill_count"),
                                                 g("sgpr_count")))
