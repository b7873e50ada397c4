"""TEST INFRASTRUCTURE ONLY — compile the reference's own Cython GIoU kernel.

Builds ``/root/reference/utils/box_intersection.pyx`` (read in place, never
copied) into ``oracle/_ref/`` so the golden-fixture generator and the
oracle self-check can call the *real* reference ``box_intersection`` (the
routine ``utils/box_util.py:691-693`` dispatches to).  The reference's own
recipe (``utils/cython_compile.py:10``) points at ``numpy/core/include``,
which does not exist under numpy 2.x, so the include path comes from
``numpy.get_include()`` here.

Output: ``oracle/_ref/box_intersection*.so`` (git-ignored; it travels to the
GPU box with the snapshot but nothing there needs it).
"""
import os
import sys

REF_PYX = "/root/reference/utils/box_intersection.pyx"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "_ref")


def build(quiet: bool = True) -> str:
    """Compile the reference Cython module; returns the _ref directory."""
    if not os.path.exists(REF_PYX):
        raise FileNotFoundError(REF_PYX)
    os.makedirs(OUT, exist_ok=True)
    import glob
    if glob.glob(os.path.join(OUT, "box_intersection*.so")):
        return OUT
    import numpy as np
    from Cython.Build import cythonize
    from setuptools import Extension
    from setuptools.dist import Distribution

    ext = Extension(
        "box_intersection",
        [REF_PYX],
        include_dirs=[np.get_include()],
        extra_compile_args=["-O2", "-w"],
    )
    exts = cythonize([ext], build_dir=os.path.join(OUT, "cy"), quiet=quiet,
                     language_level=3)
    dist = Distribution({"ext_modules": exts})
    cmd = dist.get_command_obj("build_ext")
    cmd.build_lib = OUT
    cmd.build_temp = os.path.join(OUT, "tmp")
    cmd.inplace = False
    cmd.ensure_finalized()
    cmd.run()
    return OUT


def load():
    """Import the compiled reference module (builds it if needed)."""
    d = build()
    if d not in sys.path:
        sys.path.insert(0, d)
    import box_intersection  # noqa: E402
    return box_intersection


if __name__ == "__main__":
    print(build(quiet=False))
