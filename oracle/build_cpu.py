"""Build oracle/_build/libt1dyn_cpu.so: the product dynamics header compiled for the host (g++ -fopenmp).

TEST INFRASTRUCTURE (see oracle/dyn_cpu.cpp)."""
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(HERE, "_build", "libt1dyn_cpu.so")
DEPS = [os.path.join(HERE, "dyn_cpu.cpp")] + [os.path.join(REPO, "ti5_isaacgym_amd", "csrc", f) for f in
                                              ("t1_dynamics.h", "t1_dyn5.h", "t1_common.h", "t1_model_conv.h")]


def build(force=False):
    if not force and os.path.exists(OUT) and all(os.path.getmtime(OUT) >= os.path.getmtime(d) for d in DEPS):
        return OUT
    os.makedirs(os.path.dirname(OUT), exist_ok=True)
    subprocess.run(["g++", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-std=c++17", "-o", OUT + ".tmp",
                    os.path.join(HERE, "dyn_cpu.cpp")], check=True)
    os.replace(OUT + ".tmp", OUT)
    return OUT


if __name__ == "__main__":
    print(build(force=True))
