"""Host-side mirror of the reference's renderer API over libinsitu_hip.so.

The reference host classes are Kotlin (DistributedVolumes.kt, DistributedVolumeRenderer.kt);
their GPU dispatch, texture readback and JNI exchange are what libinsitu_hip.so replaces.
`DistributedVolumes` keeps their method names and argument meaning so a caller ports 1:1:

  setVolumeDims(dims)                         DistributedVolumes.kt:142
  addVolume(volumeID, dimensions, pos, is16bit)   DistributedVolumes.kt:147  (+ model matrix)
  updateVolume(volumeID, buffer)              DistributedVolumes.kt:243
  updateData(partnerNo, numGrids, grids, origins, gridDims, domainDims)  DistributedVolumeRenderer.kt:136
  manageVDIGeneration(): one frame = render -> distributeVDIs -> composite -> gatherCompositedVDIs
                                               DistributedVolumes.kt:683-933 (here: frame())
  rotateCamera(degrees)                       DistributedVolumes.kt:779 / VolumeFromFileExample
Errors raise RuntimeError (the reference only logs, DistributedVolumes.kt:749-753).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import native, scene
from .native import check


class InSituContext:
    """One rank's libinsitu_hip context."""

    def __init__(self, width: int, height: int, *, mode: int = native.MODE_VDI, max_supersegments: int = 20,
                 bricks_per_rank: int = 1, rank: int = 0, nranks: int = 1, device: int = 0,
                 comm_id: bytes | None = None, keep_passes: bool = True, stream: int | None = None,
                 sample_cache_mb: int = 0, composite_vdi: bool = False, max_output_supersegments: int = 0,
                 local_group: "LocalGroup | None" = None, faithful: int = 0, merge_bricks: bool = False):
        self.lib = native.load()
        cfg = native.Config()
        cfg.rank, cfg.nranks, cfg.device = rank, nranks, device
        cfg.width, cfg.height = width, height
        cfg.max_supersegments = max_supersegments if mode == native.MODE_VDI else 1
        cfg.mode, cfg.bricks_per_rank = mode, bricks_per_rank
        self._comm_buf = ctypes.create_string_buffer(comm_id, native.COMM_ID_BYTES) if comm_id else None
        cfg.comm_id = ctypes.cast(self._comm_buf, ctypes.c_void_p) if comm_id else None
        cfg.stream = stream
        cfg.keep_passes = 1 if keep_passes else 0
        cfg.sample_cache_mb = sample_cache_mb
        cfg.composite_vdi = 1 if composite_vdi else 0
        cfg.max_output_supersegments = max_output_supersegments
        cfg.local_group = local_group.h if local_group is not None else None
        cfg.faithful = faithful
        cfg.merge_bricks = 1 if merge_bricks else 0
        self._group = local_group
        h = ctypes.c_void_p()
        check(self.lib.insitu_create(ctypes.byref(cfg), ctypes.byref(h)), None, "insitu_create")
        self.h = h
        self.width, self.height, self.mode = width, height, mode
        self.S = cfg.max_supersegments
        self.S_out = (max_output_supersegments or self.S) if composite_vdi else 0
        self.strip_w = width // nranks if mode == native.MODE_VDI else width
        self.rank, self.nranks, self.B = rank, nranks, bricks_per_rank

    # ---------------------------------------------------------------- lifetime
    def close(self):
        if getattr(self, "h", None):
            self.lib.insitu_destroy(self.h)
            self.h = None

    def __del__(self):  # pragma: no cover
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def _check(self, rc, what):
        check(rc, self.h, what)

    # ---------------------------------------------------------------- inputs
    def set_brick(self, slot: int, data, model_cm: np.ndarray, dtype: int | None = None):
        """data: numpy array (host) or torch tensor (host or device), index [z][y][x]."""
        ptr, on_dev, dt, keep = _buffer(data, dtype)
        if on_dev:
            # the library reads the array on its own stream: the producer (torch's current stream,
            # e.g. the simulation step) must have finished writing it
            import torch
            torch.cuda.current_stream(keep.device).synchronize()
        dims = (ctypes.c_int * 3)(int(data.shape[2]), int(data.shape[1]), int(data.shape[0]))
        model = (ctypes.c_float * 16)(*np.asarray(model_cm, dtype=np.float32).tolist())
        self._check(self.lib.insitu_set_brick(self.h, slot, ptr, dt, dims, model, 1 if on_dev else 0), "insitu_set_brick")
        del keep

    def set_transfer(self, tf: np.ndarray, cmap: np.ndarray, conv_scale: float = 1.0, conv_offset: float = 0.0):
        tf = np.ascontiguousarray(tf, dtype=np.float32)
        cmap = np.ascontiguousarray(cmap, dtype=np.float32).reshape(-1, 4)
        self._check(self.lib.insitu_set_transfer(
            self.h, tf.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), tf.size,
            cmap.ctypes.data_as(ctypes.POINTER(ctypes.c_float)), cmap.shape[0],
            ctypes.c_float(conv_scale), ctypes.c_float(conv_offset)), "insitu_set_transfer")

    # ---------------------------------------------------------------- stages
    def render(self, cam: scene.CameraSpec):
        self._cam = cam.native()
        self._check(self.lib.insitu_render(self.h, ctypes.byref(self._cam)), "insitu_render")

    def set_camera(self, cam: scene.CameraSpec):
        self._cam = cam.native()
        self._check(self.lib.insitu_set_camera(self.h, ctypes.byref(self._cam)), "insitu_set_camera")

    # ---- reference-shaped host-buffer entry points (the JNI drop-in) ----
    def distributeVDIs(self, subVDIColor: np.ndarray, subVDIDepth: np.ndarray, sizePerProcess: int, commSize: int,
                       recv: bool = True):
        """DistributedVolumes.kt:136-137 / DistributedVolumeRenderer.kt:112: all-to-all of the host sub-VDI, then
        the composite of this rank's strip.  Returns the received set (colour, depth) when recv."""
        c = np.ascontiguousarray(subVDIColor)
        d = np.ascontiguousarray(subVDIDepth)
        rc_, rd_ = (np.empty_like(c), np.empty_like(d)) if recv else (None, None)
        self._check(self.lib.insitu_distribute_vdis(
            self.h, c.ctypes.data, d.ctypes.data, int(sizePerProcess), int(commSize),
            rc_.ctypes.data if recv else None, rd_.ctypes.data if recv else None), "insitu_distribute_vdis")
        return rc_, rd_

    def gatherCompositedVDIs(self, root: int, subVDILen: int, myRank: int, commSize: int):
        """DistributedVolumeRenderer.kt:113: gather of the composited strips; root gets the image."""
        img = np.empty((self.height, self.width, 4), np.uint8) if self.rank == root else None
        self._check(self.lib.insitu_gather_composited_vdis(
            self.h, int(root), int(subVDILen), int(myRank), int(commSize),
            img.ctypes.data if img is not None else None, img.nbytes if img is not None else 0),
            "insitu_gather_composited_vdis")
        return img

    def gatherCompositedVDISet(self, compositedVDILen: int, root: int, myRank: int, commSize: int):
        """DistributedVolumes.kt:138 / :903: gather of the composited VDIs (composite_vdi contexts);
        root gets ((W,H,S_out,4) colour, (W,H,2*S_out) depth) in the reference layouts."""
        col = dep = None
        if self.rank == root:
            col = np.empty((self.width, self.height, self.S_out, 4), np.float32)
            dep = np.empty((self.width, self.height, 2 * self.S_out), np.float32)
        self._check(self.lib.insitu_gather_composited_vdi_set(
            self.h, int(compositedVDILen), int(root), int(myRank), int(commSize),
            col.ctypes.data if col is not None else None, dep.ctypes.data if dep is not None else None),
            "insitu_gather_composited_vdi_set")
        return col, dep

    def exchange(self):
        self._check(self.lib.insitu_exchange(self.h), "insitu_exchange")

    def composite(self):
        self._check(self.lib.insitu_composite(self.h), "insitu_composite")

    def gather(self, want_image: bool = True, out=None):
        """Gather the strips on rank 0; the root's (H, W, 4) rgba8 image is copied to host memory when
        want_image (into `out` when given: a uint8 numpy array or a CPU torch tensor of that shape,
        e.g. pinned, as the reference's native-owned gather buffer that streamImage receives)."""
        img = None
        if want_image and self.rank == 0:
            img = np.empty((self.height, self.width, 4), dtype=np.uint8) if out is None else out
            _check_image_out(img, self.height, self.width)
            ptr = img.data_ptr() if hasattr(img, "data_ptr") else img.ctypes.data
            nbytes = self.height * self.width * 4
            self._check(self.lib.insitu_gather(self.h, ctypes.c_void_p(ptr), nbytes), "insitu_gather")
        else:
            self._check(self.lib.insitu_gather(self.h, None, 0), "insitu_gather")
        return img

    def frame(self, cam: scene.CameraSpec, want_image: bool = False, out=None):
        self.render(cam)
        self.exchange()
        self.composite()
        return self.gather(want_image, out)

    def _image_arg(self, want_image: bool, out):
        if want_image and self.rank == 0:
            img = np.empty((self.height, self.width, 4), dtype=np.uint8) if out is None else out
            _check_image_out(img, self.height, self.width)
            ptr = img.data_ptr() if hasattr(img, "data_ptr") else img.ctypes.data
            return img, ctypes.c_void_p(ptr), self.height * self.width * 4
        return None, None, 0

    def frame_pipelined(self, cam: scene.CameraSpec, want_image: bool = False, out=None):
        """The reference's frame loop, one frame stale (DistributedVolumeRenderer.kt:530-542): render this
        camera's frame and, meanwhile, finish the previous one (exchange, composite, gather).  Returns
        (index of the completed frame or -1 on the first call, its root image or None); readbacks and
        stats() then describe that completed frame (insitu_frame_pipelined)."""
        self._cam = cam.native()
        img, ptr, n = self._image_arg(want_image, out)
        done = ctypes.c_longlong(-1)
        self._check(self.lib.insitu_frame_pipelined(self.h, ctypes.byref(self._cam), ptr, n, ctypes.byref(done)),
                    "insitu_frame_pipelined")
        return done.value, (img if done.value >= 0 else None)

    def pipeline_flush(self, want_image: bool = False, out=None):
        """Complete the pipelined frame in flight: (its index or -1 when none, its root image or None)."""
        img, ptr, n = self._image_arg(want_image, out)
        done = ctypes.c_longlong(-1)
        self._check(self.lib.insitu_pipeline_flush(self.h, ptr, n, ctypes.byref(done)), "insitu_pipeline_flush")
        return done.value, (img if done.value >= 0 else None)

    def set_option(self, option: int, value: int):
        """Tuning option (native.OPT_*) for the following renders (insitu_set_option)."""
        self._check(self.lib.insitu_set_option(self.h, int(option), int(value)), "insitu_set_option")

    def synchronize(self):
        self._check(self.lib.insitu_synchronize(self.h), "insitu_synchronize")

    # ---------------------------------------------------------------- readback
    def read(self, which: int, slot: int = 0) -> np.ndarray:
        n = self.lib.insitu_buffer_bytes(self.h, which)
        if n == 0:
            raise RuntimeError(f"buffer {which} not available")
        out = np.empty(n, dtype=np.uint8)
        self._check(self.lib.insitu_read(self.h, which, slot, out.ctypes.data, n), "insitu_read")
        W, H, S = self.width, self.height, self.S
        if which == native.BUF_VDI_COLOR:
            return out.view(np.float32).reshape(W, H, S, 4)
        if which == native.BUF_VDI_DEPTH:
            return out.view(np.float32).reshape(W, H, 2 * S)
        if which == native.BUF_OCTREE:
            return out.view(np.uint32).reshape(S, H // 8, W // 8)
        if which == native.BUF_PASSES:
            return out.reshape(H, W)
        if which in (native.BUF_PLAIN_COLOR, native.BUF_PLAIN_DEPTH):
            return out.reshape(H, W, 4)
        if which == native.BUF_IMAGE:
            return out.reshape(H, W, 4)
        if which in (native.BUF_COMPOSITED_COLOR, native.BUF_GATHERED_COLOR):
            w = self.strip_w if which == native.BUF_COMPOSITED_COLOR else W
            return out.view(np.float32).reshape(w, H, self.S_out, 4)
        if which in (native.BUF_COMPOSITED_DEPTH, native.BUF_GATHERED_DEPTH):
            w = self.strip_w if which == native.BUF_COMPOSITED_DEPTH else W
            return out.view(np.float32).reshape(w, H, 2 * self.S_out)
        if which == native.BUF_COMPOSITE_PASSES:
            return out.reshape(H, self.strip_w)
        if which == native.BUF_RECEIVED_COLOR:   # the SetOfVDI blocks, source-major
            return out.view(np.float32).reshape(-1, self.strip_w, H, S, 4)
        if which == native.BUF_RECEIVED_DEPTH:
            return out.view(np.float32).reshape(-1, self.strip_w, H, 2 * S)
        return out

    def read_columns(self, which: int, x0: int, x1: int, slot: int = 0) -> np.ndarray:
        """Columns [x0, x1) of brick `slot`'s VDI colour (nx,H,S,4), depth (nx,H,2S) or passes (H,nx)."""
        nx, H, S = x1 - x0, self.height, self.S
        shape, dt = {native.BUF_VDI_COLOR: ((nx, H, S, 4), np.float32), native.BUF_VDI_DEPTH: ((nx, H, 2 * S), np.float32),
                     native.BUF_PASSES: ((H, nx), np.uint8)}[which]
        out = np.empty(shape, dt)
        self._check(self.lib.insitu_read_region(self.h, which, slot, x0, x1, out.ctypes.data, out.nbytes),
                    "insitu_read_region")
        return out

    def stats(self) -> dict:
        st = native.Stats()
        self._check(self.lib.insitu_get_stats(self.h, ctypes.byref(st)), "insitu_get_stats")
        return {k: getattr(st, k) for k, _ in native.Stats._fields_}

    def pass_stats(self) -> tuple[float, int]:
        """(mean raymarch passes over hit rays, hit rays) of the last render."""
        m, h = ctypes.c_double(), ctypes.c_longlong()
        self._check(self.lib.insitu_pass_stats(self.h, ctypes.byref(m), ctypes.byref(h)), "insitu_pass_stats")
        return m.value, h.value

    @property
    def stream(self) -> int:
        return self.lib.insitu_stream(self.h) or 0


class LocalGroup:
    """In-process rank group (insitu_local_group): several ranks' contexts in one process exchange
    device to device instead of over RCCL -- the multi-rank data path on a single GPU.  Drive it
    stage by stage across ranks (render all, exchange all, composite all, gather all)."""

    def __init__(self, nranks: int):
        self.lib = native.load()
        h = ctypes.c_void_p()
        check(self.lib.insitu_local_group_create(nranks, ctypes.byref(h)), None, "insitu_local_group_create")
        self.h = h
        self.nranks = nranks

    def close(self):
        if getattr(self, "h", None):
            self.lib.insitu_local_group_destroy(self.h)
            self.h = None


def _check_image_out(img, height: int, width: int):
    """gather(out=...) is written as raw rgba8 through a host copy: it must be a C-contiguous uint8 array
    (numpy, or a CPU torch tensor) of shape (height, width, 4)."""
    shape = tuple(img.shape) if hasattr(img, "shape") else None
    if shape != (height, width, 4):
        raise ValueError(f"gather: out must have shape ({height}, {width}, 4), got {shape}")
    if hasattr(img, "data_ptr"):   # torch tensor
        import torch
        if img.dtype != torch.uint8 or img.device.type != "cpu" or not img.is_contiguous():
            raise ValueError("gather: out must be a contiguous uint8 CPU tensor")
    elif not (isinstance(img, np.ndarray) and img.dtype == np.uint8 and img.flags["C_CONTIGUOUS"]):
        raise ValueError("gather: out must be a C-contiguous uint8 numpy array")


def _buffer(data, dtype):
    """(pointer, on_device, insitu dtype, keepalive) of a numpy array or torch tensor."""
    try:
        import torch
    except Exception:  # pragma: no cover
        torch = None
    if torch is not None and isinstance(data, torch.Tensor):
        t = data.contiguous()
        dt = {torch.uint8: native.U8, torch.int16: native.U16, torch.uint16: native.U16,
              torch.float32: native.F32}.get(t.dtype) if dtype is None else dtype
        if dt is None:
            raise TypeError(f"unsupported tensor dtype {t.dtype}")
        return ctypes.c_void_p(t.data_ptr()), t.is_cuda, dt, t
    a = np.ascontiguousarray(data)
    dt = {np.dtype(np.uint8): native.U8, np.dtype(np.uint16): native.U16,
          np.dtype(np.float32): native.F32}.get(a.dtype) if dtype is None else dtype
    if dt is None:
        raise TypeError(f"unsupported array dtype {a.dtype}")
    return ctypes.c_void_p(a.ctypes.data), False, dt, a


class DistributedVolumes:
    """Reference-shaped host API (DistributedVolumes.kt) over InSituContext, VDI mode."""

    def __init__(self, windowWidth: int = 1280, windowHeight: int = 720, *, rank: int = 0, commSize: int = 1,
                 nodeRank: int = 0, maxSupersegments: int = 20, volumesPerRank: int = 1,
                 comm_id: bytes | None = None, generateVDIs: bool = True, compositeVDIs: bool = False,
                 maxOutputSupersegments: int = 20, basePath: str = "", dataset: str = ""):
        self.windowWidth, self.windowHeight = windowWidth, windowHeight
        self.rank, self.commSize, self.nodeRank = rank, commSize, nodeRank
        self.maxSupersegments = maxSupersegments
        self.pixelToWorld = 0.001          # DistributedVolumes.kt:106
        self.volumeDims = (0, 0, 0)
        self.volumes: dict[int, tuple] = {}
        self.maxOutputSupersegments = maxOutputSupersegments
        self.basePath, self.dataset = basePath, dataset    # dump location (DistributedVolumes.kt:507-511)
        self.cnt_sub = 0
        self.cnt_distr = 0
        self.ctx = InSituContext(windowWidth, windowHeight,
                                 mode=native.MODE_VDI if generateVDIs else native.MODE_PLAIN,
                                 max_supersegments=maxSupersegments, bricks_per_rank=volumesPerRank,
                                 rank=rank, nranks=commSize, device=nodeRank, comm_id=comm_id,
                                 composite_vdi=compositeVDIs and generateVDIs,
                                 max_output_supersegments=maxOutputSupersegments if compositeVDIs else 0)
        self.ctx.set_transfer(scene.transfer_function(), scene.colormap_hot())
        self.camera = scene.orbit_camera(windowWidth, windowHeight)
        self._yaw = 30.0
        self.vdisGathered = 0

    def setVolumeDims(self, dims):
        self.volumeDims = tuple(int(d) for d in dims)

    def addVolume(self, volumeID: int, dimensions, pos, is16bit: bool, model=None):
        if model is None:
            model = scene.brick_model(pos, self.pixelToWorld)
        self.volumes[volumeID] = (tuple(int(d) for d in dimensions), np.asarray(model, np.float32), is16bit)

    def updateVolume(self, volumeID: int, buffer):
        dims, model, is16bit = self.volumes[volumeID]
        arr = np.frombuffer(buffer, dtype=np.uint16 if is16bit else np.uint8) if isinstance(buffer, (bytes, bytearray, memoryview)) else buffer
        arr = arr.reshape(dims[2], dims[1], dims[0])
        self.ctx.set_brick(volumeID, arr, model)

    def updateData(self, partnerNo: int, numGrids: int, grids, origins, gridDims, domainDims):
        """DistributedVolumeRenderer.kt:136-160: one brick per grid of this compute partner."""
        for i in range(numGrids):
            g = gridDims[i * 6:(i + 1) * 6]
            dims = (g[3] - g[0] + 1, g[4] - g[1] + 1, g[5] - g[2] + 1)
            origin = np.asarray(origins[i * 3:(i + 1) * 3], dtype=np.float64) * 0.02   # pixelToWorld 0.02 (:361)
            self.addVolume(i, dims, origin, True, scene.brick_model(origin, 0.02))
            self.updateVolume(i, grids[i])

    def rotateCamera(self, degrees: float):
        self._yaw += degrees
        self.camera = scene.orbit_camera(self.windowWidth, self.windowHeight, yaw_deg=self._yaw)

    def manageVDIGeneration(self, frames: int = 1, want_image: bool = True, benchmarking: bool = True):
        """DistributedVolumes.kt:683-933: render -> distribute -> composite -> gather per frame.  With
        benchmarking=False the raw dumps of the reference are written (sub-VDI :848-849, composited VDI
        :894-895, frame metadata :910-915; vdi_io.py)."""
        img = None
        for _ in range(frames):
            img = self.ctx.frame(self.camera, want_image=want_image)
            if not benchmarking and self.ctx.mode == native.MODE_VDI:
                self.dumpVDIs()
            self.vdisGathered += 1
        return img

    def dumpVDIs(self):
        """The reference's non-benchmarking dumps of one frame: sub-VDI (:848-849) with its octree grid
        (VolumeFromFileExample.kt:1067), the received set (SetOfVDI, :974-975), the composited VDI
        (:894-895) and the frame metadata (:910-915)."""
        from . import vdi_io
        sub = vdi_io.vdi_paths(self.basePath, self.dataset, "SubVDI", self.cnt_sub)
        paths = list(vdi_io.write_vdi(self.basePath, self.dataset, "SubVDI", self.cnt_sub,
                                      self.ctx.read(native.BUF_VDI_COLOR), self.ctx.read(native.BUF_VDI_DEPTH)))
        paths.append(vdi_io.write_octree(str(sub[0])[:-len("_col")] + "_octree", self.ctx.read(native.BUF_OCTREE)))
        paths += vdi_io.write_received_set(self.basePath, self.dataset, self.cnt_distr,
                                           self.ctx.read(native.BUF_RECEIVED_COLOR),
                                           self.ctx.read(native.BUF_RECEIVED_DEPTH))
        self.cnt_distr += 1
        if self.ctx.S_out:
            paths += vdi_io.write_vdi(self.basePath, self.dataset, "CompositedVDI", self.cnt_sub,
                                      self.ctx.read(native.BUF_COMPOSITED_COLOR),
                                      self.ctx.read(native.BUF_COMPOSITED_DEPTH))
        dims, model, _ = self.volumes.get(0, (self.volumeDims, np.eye(4, dtype=np.float32).reshape(16), False))
        paths.append(vdi_io.write_metadata(self.basePath, self.dataset, self.windowWidth, self.windowHeight,
                                           self.maxSupersegments, self.vdisGathered, self.camera, model, dims))
        self.cnt_sub += 1
        return paths
