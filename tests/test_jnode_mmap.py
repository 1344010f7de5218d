"""JNodeTable's mapped storage (sheep_amd/lib/jnode.h, the reference's State::MAPPED,
jnode.cpp:52-110): build into a mapped .tre, reopen in place, save — byte-equal to the heap
table's file.  Host code only (g++), no GPU call."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_jnode_mapped_storage(tmp_path):
    exe = tmp_path / "jnode_mmap"
    subprocess.run(["g++", "-O1", "-std=c++17", "-Wall", "-I", os.path.join(ROOT, "include"),
                    "-I", os.path.join(ROOT, "sheep_amd", "lib"), "-o", str(exe),
                    os.path.join(ROOT, "tests", "cpp", "jnode_mmap.cpp"),
                    "-L", os.path.join(ROOT, "sheep_amd"), "-lsheep_amd",
                    "-Wl,-rpath," + os.path.join(ROOT, "sheep_amd")], check=True)
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True)
    assert out.returncode == 0, out.stderr
    assert out.stdout.strip() == "ok"
