"""Import the reference's own Python modules in THIS container (fixture generation only).

Recipe of SURVEY.md §8c: stub the import-time-only dependencies that are
absent here (plyfile, trimesh, cv2, imageio, torchvision, detectron2.structures),
inject the oracle's CPU ``third_party.pointnet2`` restatement, compile the
reference Cython GIoU into ``oracle/_ref`` and load ``models/*.py`` under a
synthetic ``models`` package (``models/__init__.py`` eagerly imports the
RegionCLIP/detectron2 builder).  Nothing here runs on the GPU box:
``/root/reference`` does not exist there; the fixtures this produces are
committed under ``tests/golden``.
"""
import importlib.util
import os
import sys
import types

REF = "/root/reference"
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _stub(name, **attrs):
    m = types.ModuleType(name)
    for k, v in attrs.items():
        setattr(m, k, v)
    sys.modules[name] = m
    return m


class _Holder:
    def __init__(self, *a, **kw):
        self.args = a
        self.__dict__.update(kw)


class Boxes:
    """Stand-in for detectron2.structures.Boxes (a plain (N,4) holder)."""

    def __init__(self, tensor):
        self.tensor = tensor


class Instances:
    """Stand-in for detectron2.structures.Instances (image_size + fields)."""

    def __init__(self, image_size, **kwargs):
        self.image_size = image_size
        self._fields = dict(kwargs)

    def __getattr__(self, k):
        f = self.__dict__.get("_fields", {})
        if k in f:
            return f[k]
        raise AttributeError(k)


_LOADED = {}


def load_reference():
    if _LOADED:
        return _LOADED
    sys.dont_write_bytecode = True
    _stub("plyfile", PlyData=_Holder, PlyElement=_Holder)
    _stub("trimesh")
    _stub("cv2")
    _stub("imageio", imread=lambda *a, **k: None)
    tv = _stub("torchvision")
    tvt = _stub("torchvision.transforms", InterpolationMode=types.SimpleNamespace(BICUBIC=3))
    tv.transforms = tvt
    d2 = _stub("detectron2")
    d2s = _stub("detectron2.structures", Boxes=Boxes, Instances=Instances)
    d2.structures = d2s
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    from oracle import pointnet2_ref, build_ref
    pointnet2_ref.install_as_third_party()
    bi = build_ref.load()
    if REF not in sys.path:
        sys.path.insert(0, REF)
    import utils  # noqa: F401  (reference utils package)
    sys.modules["utils.box_intersection"] = bi
    import utils.box_util as box_util
    assert box_util.box_intersection is not None, "Cython GIoU not picked up"
    import utils.nms as nms
    import utils.pc_util as pc_util
    import utils.image_util as image_util
    import utils.misc as misc
    # models package without its eager __init__
    pkg = types.ModuleType("models")
    pkg.__path__ = [os.path.join(REF, "models")]
    sys.modules["models"] = pkg
    mods = {}
    for name in ("helpers", "position_embedding", "transformer", "model_3detr"):
        spec = importlib.util.spec_from_file_location(f"models.{name}",
                                                      os.path.join(REF, "models", f"{name}.py"))
        m = importlib.util.module_from_spec(spec)
        sys.modules[f"models.{name}"] = m
        spec.loader.exec_module(m)
        setattr(pkg, name, m)
        mods[name] = m
    spec = importlib.util.spec_from_file_location("ref_criterion", os.path.join(REF, "criterion.py"))
    crit = importlib.util.module_from_spec(spec)
    sys.modules["ref_criterion"] = crit
    spec.loader.exec_module(crit)
    import datasets.sunrgbd as sunrgbd  # noqa: E402
    _LOADED.update(dict(box_util=box_util, nms=nms, pc_util=pc_util, image_util=image_util,
                        misc=misc, criterion=crit, sunrgbd=sunrgbd, box_intersection=bi, **mods))
    return _LOADED


if __name__ == "__main__":
    r = load_reference()
    print(sorted(r))
