"""Scene inputs of the in-situ path: camera matrices, brick model matrices, transfer
function, colour map and synthetic simulation volumes.

These replace what scenery computes on the JVM side for the shaders:
  * projection: JOML Matrix4f.perspective(fov, aspect, near, far) followed by the Vulkan
    coordinate fix of DistributedVolumes.kt:67-79 (y flipped, z remapped to [0,1]);
  * view: the camera's getTransformation() (a look-at matrix);
  * model: Volume position + pixelToWorldRatio with Origin.FrontBottomLeft
    (DistributedVolumes.kt:160-165, DistributedVolumeRenderer.kt:351-369);
  * transfer function: piecewise-linear control points sampled into a 1024-texel LUT
    (control points of DistributedVolumeRenderer.kt:374-380);
  * colour map: "hot" (DistributedVolumeRenderer.kt:333), 256 texels.
All matrices are float32, column-major flattened (GLSL/JOML order).
"""
from __future__ import annotations

import math

import numpy as np

VULKAN_FIX = np.array([[1.0, 0.0, 0.0, 0.0],
                       [0.0, -1.0, 0.0, 0.0],
                       [0.0, 0.0, 0.5, 0.5],
                       [0.0, 0.0, 0.0, 1.0]])   # row-major form of DistributedVolumes.kt:67-72

NEAR, FAR = 0.1, 20.0   # DistributedVolumes.kt:484-485; VDIGenerator.comp:241-242


def col_major(m: np.ndarray) -> np.ndarray:
    """row-major 4x4 (float64) -> column-major float32[16]"""
    return np.ascontiguousarray(np.asarray(m, dtype=np.float64).T.reshape(16).astype(np.float32))


def perspective(fov_deg: float, aspect: float, near: float = NEAR, far: float = FAR) -> np.ndarray:
    """JOML Matrix4f.perspective (OpenGL clip space), row-major float64."""
    h = math.tan(math.radians(fov_deg) * 0.5)
    m = np.zeros((4, 4))
    m[0, 0] = 1.0 / (h * aspect)
    m[1, 1] = 1.0 / h
    m[2, 2] = (far + near) / (near - far)
    m[2, 3] = (far + far) * near / (near - far)
    m[3, 2] = -1.0
    return m


def look_at(eye, target, up=(0.0, 1.0, 0.0)) -> np.ndarray:
    eye, target, up = (np.asarray(v, dtype=np.float64) for v in (eye, target, up))
    f = target - eye
    f /= np.linalg.norm(f)
    s = np.cross(f, up)
    s /= np.linalg.norm(s)
    u = np.cross(s, f)
    m = np.eye(4)
    m[0, :3], m[1, :3], m[2, :3] = s, u, -f
    m[0, 3], m[1, 3], m[2, 3] = -s @ eye, -u @ eye, f @ eye
    return m


class CameraSpec:
    """View/projection of one frame plus the sampling step `nw`."""

    def __init__(self, view: np.ndarray, proj_gl: np.ndarray, nw: float, fwnw: float = 0.0, tmax: float = 1.0):
        self.view_rm = np.asarray(view, dtype=np.float64)
        self.proj_rm = VULKAN_FIX @ np.asarray(proj_gl, dtype=np.float64)
        self.view = col_major(self.view_rm)
        self.proj = col_major(self.proj_rm)
        self.inv_view = col_major(np.linalg.inv(self.view_rm))
        self.inv_proj = col_major(np.linalg.inv(self.proj_rm))
        self.nw = np.float32(nw)
        self.fwnw = np.float32(fwnw)
        self.tmax = np.float32(tmax)

    def native(self):
        from .native import Camera, F16
        c = Camera()
        c.view = F16(*self.view.tolist())
        c.proj = F16(*self.proj.tolist())
        c.inv_view = F16(*self.inv_view.tolist())
        c.inv_proj = F16(*self.inv_proj.tolist())
        c.has_inverses = 1
        c.nw, c.fwnw, c.tmax = float(self.nw), float(self.fwnw), float(self.tmax)
        return c


def ray_length(cam: CameraSpec) -> float:
    """|wback - wfront| of the centre ray (world units)."""
    ipv = np.linalg.inv(cam.proj_rm @ cam.view_rm)
    f = ipv @ np.array([0.0, 0.0, -1.0, 1.0])
    b = ipv @ np.array([0.0, 0.0, 1.0, 1.0])
    return float(np.linalg.norm(b[:3] / b[3] - f[:3] / f[3]))


def orbit_camera(width: int, height: int, center=(0.0, 0.0, 0.0), radius: float = 3.5, yaw_deg: float = 30.0,
                 pitch_deg: float = 20.0, fov_deg: float = 50.0, voxel_world: float = 2.0 / 1024.0,
                 samples_per_voxel: float = 1.0) -> CameraSpec:
    """Camera on a sphere around `center` looking at it, with nw chosen so
    that the step along the centre ray is voxel_world/samples_per_voxel."""
    yaw, pitch = math.radians(yaw_deg), math.radians(pitch_deg)
    c = np.asarray(center, dtype=np.float64)
    eye = c + radius * np.array([math.cos(pitch) * math.sin(yaw), math.sin(pitch), math.cos(pitch) * math.cos(yaw)])
    view = look_at(eye, c)
    cam = CameraSpec(view, perspective(fov_deg, width / height), nw=1.0)
    cam.nw = np.float32(voxel_world / samples_per_voxel / ray_length(cam))
    return cam


def brick_model(origin_world, voxel_world: float) -> np.ndarray:
    """World matrix of a brick: world = origin + voxel_world * p (p in voxel space)."""
    m = np.eye(4)
    m[0, 0] = m[1, 1] = m[2, 2] = voxel_world
    m[:3, 3] = np.asarray(origin_world, dtype=np.float64)
    return col_major(m)


def inverse_model(model_cm: np.ndarray) -> np.ndarray:
    """float32 inverse of a column-major model matrix, computed in float64 (as the library does)."""
    m = np.asarray(model_cm, dtype=np.float64).reshape(4, 4).T
    return col_major(np.linalg.inv(m))


def transfer_function(points=((0.0, 0.0), (0.2, 0.1), (0.4, 0.4), (0.8, 0.6), (1.0, 0.75)), n: int = 1024) -> np.ndarray:
    """Piecewise-linear alpha LUT sampled at texel centres (scenery TransferFunction)."""
    xs = np.array([p[0] for p in points], dtype=np.float64)
    ys = np.array([p[1] for p in points], dtype=np.float64)
    t = (np.arange(n) + 0.5) / n
    return np.interp(t, xs, ys).astype(np.float32)


def colormap_hot(n: int = 256) -> np.ndarray:
    """'hot' colour map: black -> red -> yellow -> white, alpha 1, as n x 4 float32."""
    t = (np.arange(n) + 0.5) / n
    r = np.clip(t / 0.375, 0.0, 1.0)
    g = np.clip((t - 0.375) / 0.375, 0.0, 1.0)
    b = np.clip((t - 0.75) / 0.25, 0.0, 1.0)
    return np.stack([r, g, b, np.ones_like(t)], axis=1).astype(np.float32)


def folded_conv_scale(conv_scale: float, dtype: int) -> np.float32:
    """conv_scale with the unorm normalisation folded in, rounded exactly as the library does."""
    from .native import U8, U16
    norm = np.float32(1.0) / np.float32(255.0) if dtype == U8 else (
        np.float32(1.0) / np.float32(65535.0) if dtype == U16 else np.float32(1.0))
    return np.float32(np.float32(conv_scale) * norm)


# ---------------------------------------------------------------- synthetic volumes

def gray_scott(n: int, steps: int = 1500, seed: int = 1000, F: float = 0.03, k: float = 0.055, Du: float = 0.2,
               Dv: float = 0.1, dt: float = 0.8, device: str = "cpu", sim_n: int | None = None):
    """3-D Gray-Scott reaction-diffusion (periodic, explicit Euler), u=1, v=0 plus random seed
    cubes (seed 1000 as VDIGenerationExample.kt:186).  Returns v as a float32 torch tensor
    (n,n,n), index [z,y,x].

    Simulated on a sim_n^3 grid (default min(n, 128), at least 64: smaller grids lose every
    seed) and resampled trilinearly to n^3.  dt = 0.8 keeps Du*dt*6 < 1 (explicit stability);
    F=0.03, k=0.055 is the spot/worm regime that survives in 3-D (SURVEY.md's F=0.04, k=0.06
    decays to v = 0 at these sizes)."""
    import torch
    m = sim_n if sim_n is not None else max(64, min(n, 128))
    g = torch.Generator(device="cpu").manual_seed(seed)
    u = torch.ones((m, m, m), dtype=torch.float32)
    v = torch.zeros((m, m, m), dtype=torch.float32)
    size = max(3, m // 10)
    for _ in range(max(8, (m // 8) ** 2 // 2)):
        z, y, x = (int(t) for t in torch.randint(0, m - size, (3,), generator=g))
        u[z:z + size, y:y + size, x:x + size] = 0.5
        v[z:z + size, y:y + size, x:x + size] = 0.25
    u, v = u.to(device), v.to(device)

    if u.is_cuda:   # one fused HIP kernel per step (libinsitu_sim.so): same formula, ~25x faster
        _sim_gray_scott_device(u, v, steps, F, k, Du, Dv, dt)
        return v if m == n else resample(v, n)

    def lap(a):
        return (torch.roll(a, 1, 0) + torch.roll(a, -1, 0) + torch.roll(a, 1, 1) + torch.roll(a, -1, 1)
                + torch.roll(a, 1, 2) + torch.roll(a, -1, 2) - 6.0 * a)

    for _ in range(steps):
        uvv = u * v * v
        u = u + dt * (Du * lap(u) - uvv + F * (1.0 - u))
        v = v + dt * (Dv * lap(v) + uvv - (F + k) * v)
    return v if m == n else resample(v, n)


_SIM_LIB = None


def _sim_gray_scott_device(u, v, steps, F, k, Du, Dv, dt):
    """The explicit-Euler loop of gray_scott on the GPU (csrc/sim_gray_scott.hip, libinsitu_sim.so), in
    place on the contiguous float32 device tensors u, v.  Synthetic input only (the OpenFPM simulation's
    stand-in), not the rendering path."""
    import ctypes
    from pathlib import Path

    import torch
    global _SIM_LIB
    if _SIM_LIB is None:
        path = Path(__file__).resolve().parent.parent / "lib" / "libinsitu_sim.so"
        if not path.exists():
            raise RuntimeError(f"{path} not found: build it with `make -C scenery-insitu_amd`")
        lib = ctypes.CDLL(str(path))
        fp, i, f = ctypes.c_void_p, ctypes.c_int, ctypes.c_float
        lib.insitu_sim_gray_scott.argtypes = [fp, fp, fp, fp, i, i, f, f, f, f, f, fp]
        lib.insitu_sim_gray_scott.restype = i
        _SIM_LIB = lib
    u2, v2 = torch.empty_like(u), torch.empty_like(v)
    stream = torch.cuda.current_stream(u.device).cuda_stream
    rc = _SIM_LIB.insitu_sim_gray_scott(u.data_ptr(), v.data_ptr(), u2.data_ptr(), v2.data_ptr(), u.shape[0], steps,
                                        F, k, Du, Dv, dt, stream)
    if rc != 0:
        raise RuntimeError(f"insitu_sim_gray_scott failed ({rc})")


def resample(vol, n_out: int):
    """Trilinear resampling of a (n,n,n) torch tensor to (n_out,n_out,n_out)."""
    import torch
    return torch.nn.functional.interpolate(vol[None, None], size=(n_out, n_out, n_out), mode="trilinear",
                                           align_corners=True)[0, 0].contiguous()


def to_uint16(vol, vmax: float = 0.5):
    """round(clamp(v/vmax)*65535) as uint16 numpy (parity inputs are uint16)."""
    a = np.asarray(vol.detach().cpu().numpy() if hasattr(vol, "detach") else vol, dtype=np.float64)
    return np.round(np.clip(a / vmax, 0.0, 1.0) * 65535.0).astype(np.uint16)


def grid_bricks(n_global: int, bricks_per_axis: int = 2, world: float = 2.0):
    """(origin_world, voxel_world, brick_index_xyz) of the bricks of a cube [-1,1]^3 split
    bricks_per_axis^3 ways (config 2: 2x2x2 bricks of 512^3 = 1024^3 global)."""
    nb = n_global // bricks_per_axis
    vw = world / n_global
    out = []
    for bz in range(bricks_per_axis):
        for by in range(bricks_per_axis):
            for bx in range(bricks_per_axis):
                origin = (-world / 2 + bx * nb * vw, -world / 2 + by * nb * vw, -world / 2 + bz * nb * vw)
                out.append((origin, vw, (bx, by, bz)))
    return out


def vortex_ring(n: int, z0: int = 0, nz: int | None = None, radius: float = 0.25, core: float = 0.05,
                seed: int = 1000, modes: int = 4, amplitude: float = 0.06, device: str = "cpu"):
    """Vorticity magnitude |w| of a perturbed vortex ring on an n^3 grid of the unit cube (config 3,
    SURVEY.md 8d: Gaussian tube, radius 0.25, core 0.05, seed 1000), z-rows [z0, z0+nz) only, so
    that each rank builds just its own slab.  Float32 torch tensor (nz, n, n), index [z, y, x].

    The ring lies in the x-z plane around the cube centre, its radius and height perturbed by
    `modes` azimuthal waves with seeded amplitudes and phases; |w| = exp(-d^2 / core^2) with d the
    distance to the perturbed centre line (Lamb-Oseen core, peak 1).  The centre line is
    approximated by the nearest point at the voxel's own azimuth, which is exact for the
    unperturbed ring and within O(amplitude^2) otherwise (a synthetic field, not a solver)."""
    import torch
    nz = n - z0 if nz is None else nz
    g = torch.Generator(device="cpu").manual_seed(seed)
    amp_r = (torch.rand(modes, generator=g, dtype=torch.float64) * 2.0 - 1.0) * amplitude
    amp_h = (torch.rand(modes, generator=g, dtype=torch.float64) * 2.0 - 1.0) * amplitude
    ph_r = torch.rand(modes, generator=g, dtype=torch.float64) * (2.0 * math.pi)
    ph_h = torch.rand(modes, generator=g, dtype=torch.float64) * (2.0 * math.pi)
    c = (torch.arange(n, dtype=torch.float32, device=device) + 0.5) / n - 0.5
    cz = (torch.arange(z0, z0 + nz, dtype=torch.float32, device=device) + 0.5) / n - 0.5
    z = cz.view(nz, 1, 1)
    y = c.view(1, n, 1)
    x = c.view(1, 1, n)
    phi = torch.atan2(z, x)                                   # (nz, 1, n)
    rr = torch.full_like(phi, radius)
    hh = torch.zeros_like(phi)
    for m in range(modes):
        rr = rr + float(amp_r[m]) * radius * torch.cos((m + 2) * phi + float(ph_r[m]))
        hh = hh + float(amp_h[m]) * radius * torch.cos((m + 2) * phi + float(ph_h[m]))
    rho = torch.sqrt(x * x + z * z)                           # distance from the ring axis (y)
    d2 = (rho - rr) ** 2 + (y - hh) ** 2                      # (nz, n, n)
    return torch.exp(-d2 / (core * core)).to(torch.float32).contiguous()


def slab_bricks(n_global: int, nslabs: int, world: float = 2.0):
    """(origin_world, voxel_world, (z0, nz)) of the z-slabs of an n_global^3 grid over the cube
    [-1,1]^3 (config 3: the global grid slab-decomposed over the ranks, one slab per rank)."""
    if n_global % nslabs:
        raise ValueError(f"{n_global} rows do not split into {nslabs} slabs")
    nz = n_global // nslabs
    vw = world / n_global
    return [((-world / 2, -world / 2, -world / 2 + s * nz * vw), vw, (s * nz, nz)) for s in range(nslabs)]
