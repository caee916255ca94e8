"""Scene model mirroring the reference's host API.

Reference types and where they live:
  material::lambert / metal / dielectric      src/material.hxx:12-39
  material::types (variant)                   src/material.hxx:41-51
  primitives::sphere                          src/primitives.hxx:6-17
  raytracer::data {spheres, materials}        src/raytracer.hxx:19-30
  scene construction in main()                src/main.cxx:120-177

`RaytracerData` keeps the reference's push_back/emplace_back style so code written against
the reference reads the same; `.arrays()` packs it into the C-ABI records (include/rt_api.h).
"""
import ctypes as C
from dataclasses import dataclass

import numpy as np

from . import _abi as abi
from ._lib import check, lib


@dataclass(frozen=True)
class Lambert:
    """material::lambert{albedo} (src/material.hxx:12-19)."""
    albedo: tuple = (1.0, 1.0, 1.0)


@dataclass(frozen=True)
class Metal:
    """material::metal{albedo, roughness} (src/material.hxx:21-29)."""
    albedo: tuple = (1.0, 1.0, 1.0)
    roughness: float = 0.0


@dataclass(frozen=True)
class Dielectric:
    """material::dielectric{albedo, refraction_index} (src/material.hxx:31-39)."""
    albedo: tuple = (1.0, 1.0, 1.0)
    refraction_index: float = 1.0


@dataclass(frozen=True)
class Sphere:
    """primitives::sphere{center, radius, material_index} (src/primitives.hxx:6-17)."""
    center: tuple
    radius: float
    material_index: int


def _vec3(v):
    if np.isscalar(v):
        v = (v, v, v)  # math::vec3{s} broadcasts (src/math.hxx:74-76)
    return tuple(float(np.float32(x)) for x in v)


class RaytracerData:
    """raytracer::data: the sphere list and the material list (src/raytracer.hxx:19-30).

    The reference's bounce bound (bounces_number = 64) and its RNG are render parameters
    here (`max_depth`, `seed` of render_*), not scene state.
    """

    bounces_number = 64

    def __init__(self, spheres=None, materials=None):
        self.spheres = list(spheres or [])
        self.materials = list(materials or [])

    # ---- reference-style construction ------------------------------------------------
    def add_material(self, m):
        self.materials.append(m)
        return len(self.materials) - 1

    def add_sphere(self, center, radius, material_index):
        self.spheres.append(Sphere(_vec3(center), float(np.float32(radius)), int(material_index)))

    # ---- packing ---------------------------------------------------------------------
    def arrays(self):
        """(spheres, materials) as numpy record arrays in the C-ABI layout."""
        s = np.zeros(len(self.spheres), dtype=abi.SPHERE_DTYPE)
        for i, sp in enumerate(self.spheres):
            s[i] = (sp.center, sp.radius, sp.material_index)
        m = np.zeros(len(self.materials), dtype=abi.MATERIAL_DTYPE)
        for i, mt in enumerate(self.materials):
            if isinstance(mt, Lambert):
                m[i] = (abi.RT_LAMBERT, _vec3(mt.albedo), 0.0)
            elif isinstance(mt, Metal):
                m[i] = (abi.RT_METAL, _vec3(mt.albedo), mt.roughness)
            elif isinstance(mt, Dielectric):
                m[i] = (abi.RT_DIELECTRIC, _vec3(mt.albedo), mt.refraction_index)
            else:
                raise TypeError(f"unsupported material type {type(mt).__name__}")  # raytracer.hxx:196
        return s, m

    @classmethod
    def from_arrays(cls, spheres, materials):
        d = cls()
        for rec in materials:
            k, alb, p = int(rec["kind"]), tuple(float(x) for x in rec["albedo"]), float(rec["param"])
            d.materials.append(Lambert(alb) if k == abi.RT_LAMBERT else Metal(alb, p) if k == abi.RT_METAL
                               else Dielectric(alb, p))
        for rec in spheres:
            d.spheres.append(Sphere(tuple(float(x) for x in rec["center"]), float(rec["radius"]),
                                    int(rec["material"])))
        return d


def _from_c(fn, *pre):
    ns, nm = C.c_uint32(0), C.c_uint32(0)
    check(fn(*pre, None, 0, C.byref(ns), None, 0, C.byref(nm)))
    s = np.zeros(ns.value, dtype=abi.SPHERE_DTYPE)
    m = np.zeros(nm.value, dtype=abi.MATERIAL_DTYPE)
    check(fn(*pre, abi.ptr(s, C.POINTER(abi.RtSphere)), len(s), C.byref(ns),
             abi.ptr(m, C.POINTER(abi.RtMaterial)), len(m), C.byref(nm)))
    return s, m


def simple_scene_arrays():
    """The reference's scene (src/main.cxx:120-129) as C-ABI records."""
    return _from_c(lib().rt_scene_simple)


def huge_scene_arrays(seed=1234):
    """The reference's random-sphere scene (src/main.cxx:131-177) for std::mt19937{seed}."""
    return _from_c(lib().rt_scene_huge, seed)


def cuda_scene_arrays():
    """The reference CUDA variant's hardcoded scene (src/CUDA/cuda_impl.cu:425-437)."""
    return _from_c(lib().rt_scene_cuda)


def simple_scene():
    return RaytracerData.from_arrays(*simple_scene_arrays())


def huge_scene(seed=1234):
    return RaytracerData.from_arrays(*huge_scene_arrays(seed))
