"""Multi-GPU frame tiling: one process per GPU, rows dealt in block-cyclic bands,
assembled on rank 0 with one RCCL gather over xGMI.

The reference renders serially on one core (src/render.rs:32-37) and has no
distributed path; this is the MI355X-native scale-out of that loop.  Pixels are
independent, so the only exchange step is assembling the frame:

  band b (rows [b*B, (b+1)*B)) belongs to rank b % world       (load balance: costly
  glass-sphere rows are spread over every rank)
  each rank renders its bands back to back into a [rows_per_rank, W, 3] buffer
  torch.distributed.gather (backend "nccl" == RCCL) -> rank 0: [world, rows_per_rank, W, 3]
  rank 0: HIP unpermute kernel -> row-major [H, W, 3] frame
"""
import torch
import torch.distributed as dist

from . import DeviceScene, RtError, abi, band_rows_per_rank, unpermute_bands_batch_async


def band_rows_per_rank_py(y_res, band_rows, world):
    """Pure-Python statement of rt_band_rows_per_rank (include/rt_api.h)."""
    n_bands = (y_res + band_rows - 1) // band_rows
    return ((n_bands + world - 1) // world) * band_rows


def local_rows(y_res, band_rows, rank, world):
    """Global row index of each local row of `rank` (-1 for padding)."""
    rpr = band_rows_per_rank_py(y_res, band_rows, world)
    rows = []
    for lr in range(rpr):
        band = lr // band_rows
        v = (band * world + rank) * band_rows + (lr - band * band_rows)
        rows.append(v if v < y_res else -1)
    return rows


class FrameTiler:
    """Renders this rank's share of a frame and gathers the frame on rank 0."""

    def __init__(self, scene: DeviceScene, width, height, depth, band_rows=8, rank=0, world=1,
                 device=None, spp=1, seed=0, batch=1, rgb8=False, force_gather=False, split=False,
                 frames_out=None, band_out=None, no_gather=False):
        """rgb8: render and gather only Color::as_u8 bytes (3 B per pixel instead of 12; the
        level-0 combine writes them, rt_render_bands_ex_async with no float buffer).
        force_gather: at world 1 too, assemble through the process group's gather and the
        un-permute kernel (a one-rank communicator: runs the RCCL exchange on one GPU).
        split: at world 1, single frames (batch 1, spp 1, f32) go through rt_render_frame_async
        -- rt_render's two band shares side by side, stream-ordered -- instead of one pass
        (render on a created torch stream, not the null stream: rt_api.h).
        frames_out: a [batch, H, W, 3] tensor of whole frames this tiler's rank (a band share of
        one device, world = the shares) fills in place (rt_render_bands_direct_async); the
        other shares fill the rest of the same frames, and nothing is gathered.
        band_out: a [batch, rows_per_rank, W, 3] tensor (a slice of a caller's buffer) that
        receives this rank's band buffers; the caller assembles them (FramePipeline's gathered
        band-share groups), this tiler never gathers.
        no_gather: render this rank's bands of a world > 1 frame without any exchange (one
        GPU standing in for one rank of an N-GPU run: tools/scale_projection.py)."""
        self.scene = scene
        self.rgb8 = bool(rgb8) and spp == 1
        self.spp, self.seed = spp, seed
        self.w, self.h, self.depth = width, height, depth
        self.band_rows, self.rank, self.world = band_rows, rank, world
        self.direct = frames_out is not None
        if self.direct and (spp != 1 or force_gather or split):
            raise ValueError("frames_out: spp 1, no gather, no split")
        self.external = band_out is not None
        self.gather = not no_gather and not self.direct and not self.external and (world > 1 or bool(force_gather))
        self.split = bool(split) and not self.gather and spp == 1 and not self.rgb8 and int(batch) == 1
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.rpr = band_rows_per_rank(height, band_rows, world)
        assert self.rpr == band_rows_per_rank_py(height, band_rows, world)
        # frames per pipeline pass (rt_render_bands_batch_async; 1 = rt_render_bands_async)
        self.batch = max(1, min(int(batch), int(abi.lib().rt_max_frames())))
        if spp > 1:
            self.batch = 1
        self.cam = abi.camera(width, height)
        dt = torch.uint8 if self.rgb8 else torch.float32
        if self.direct:
            assert tuple(frames_out.shape) == (self.batch, height, width, 3) and frames_out.dtype == dt
            assert frames_out.is_contiguous() and frames_out.device == self.device
            self.locals = frames_out
        elif self.external:
            assert tuple(band_out.shape) == (self.batch, self.rpr, width, 3) and band_out.dtype == dt
            assert band_out.is_contiguous() and band_out.device == self.device
            self.locals = band_out
        else:
            self.locals = torch.zeros((self.batch, self.rpr, width, 3), dtype=dt, device=self.device)
        self.local = self.locals[0]
        self.counters = torch.zeros(3, dtype=torch.int64, device=self.device)
        self.gathered = None
        self.frames = None          # [batch, H, W, 3]: the last pass's assembled frames (rank 0)
        if rank == 0 and self.gather:
            # one gather per pass: every rank's `batch` band buffers, rank-major
            self.gathered = torch.zeros((world, self.batch, self.rpr, width, 3), dtype=dt, device=self.device)
            self.frames = torch.zeros((self.batch, height, width, 3), dtype=dt, device=self.device)
        elif not self.gather and not self.external:
            self.frames = self.locals[:, :height]
        self.frame = self.frames[0] if self.frames is not None else None
        self.last = 1               # frames in the last pass
        self.last_cams = [self.cam]  # their cameras

    def render_local(self, n=1, cams=None):
        """Render n (<= batch) frames of this rank's bands on the current stream; cams: their
        cameras (default: Camera::new for every frame)."""
        stream = torch.cuda.current_stream(self.device).cuda_stream
        self.last = n
        assert n <= self.batch
        cams = list(cams) if cams is not None else [self.cam] * n
        self.last_cams = cams
        if self.direct:
            ptr = self.locals.data_ptr()
            self.scene.render_bands_direct_async(cams, self.depth, self.band_rows, self.rank, self.world,
                                                 0 if self.rgb8 else ptr, ptr if self.rgb8 else 0,
                                                 self.counters.data_ptr(), stream)
        elif self.rgb8:
            self.scene.render_bands_ex_async(cams, self.depth, self.band_rows, self.rank, self.world, 0,
                                             self.locals.data_ptr(), self.counters.data_ptr(), stream)
        elif n == 1 and self.split:  # the frame's rows land row-major at the buffer's start
            self.scene.render_frame_async(cams[0], self.depth, self.local.data_ptr(), self.counters.data_ptr(), stream)
        elif n == 1:
            self.scene.render_bands_async(cams[0], self.depth, self.band_rows, self.rank, self.world,
                                          self.local.data_ptr(), self.counters.data_ptr(), stream,
                                          spp=self.spp, seed=self.seed)
        else:
            self.scene.render_bands_batch_async(cams, self.depth, self.band_rows, self.rank,
                                                self.world, self.locals.data_ptr(), self.counters.data_ptr(),
                                                stream)

    def assemble(self):
        """Gather every rank's bands of the last pass's frames on rank 0 -- one gather for the
        whole pass -- and restore row order, every frame of the pass in one launch (no-op at
        world 1 unless force_gather)."""
        if not self.gather:
            return self.frame
        stream = torch.cuda.current_stream(self.device).cuda_stream
        n = self.last
        local = self.locals[:n]
        if dist.get_backend() == "gloo":
            # CPU rehearsal of the exchange (several ranks sharing one GPU); RCCL runs the
            # same gather directly on device buffers
            host = local.cpu()
            glist = [torch.empty_like(host) for _ in range(self.world)] if self.rank == 0 else None
            dist.gather(host, gather_list=glist, dst=0)
            if self.rank == 0:
                for r in range(self.world):
                    self.gathered[r, :n].copy_(glist[r])
        else:
            glist = [self.gathered[r, :n] for r in range(self.world)] if self.rank == 0 else None
            dist.gather(local, gather_list=glist, dst=0)
        if self.rank == 0:
            unpermute_bands_batch_async(self.gathered.data_ptr(), self.w, self.h, self.band_rows, self.world, n,
                                        self.batch, self.frames.data_ptr(), stream, rgb8=self.rgb8)
        return self.frame

    def step(self):
        self.render_local()
        return self.assemble()


class FramePipeline:
    """Consecutive frames with `inflight` frames in flight (DESIGN.md "Frames in flight").

    Slot i = its own scene handle (slot 0 the caller's, the others rt_scene_clone: each its
    own workspace; one handle never runs two renders at once, mirroring the reference's
    !Sync Scene) + its own HIP stream + its own FrameTiler.  Pass k renders on slot k % inflight.  At world > 1 each pass's
    gather + un-permute runs on the caller's stream once its slot is done, and the slot's
    next render waits on an event recorded after that gather (the gather reads the slot's
    band buffer).  Every frame is rendered and gathered in full.

    sub_bands S > 1: the slots form inflight / S groups of S band shares; pass k's frames go to
    group k % groups, whose S slots each render their share of the rows of every frame of the
    pass.  A pass then mixes S times as many frames as a whole-frame pass with the same rays
    in flight -- more rays from the same place per wave (DESIGN.md "Band-share slot groups").
    At world 1 the shares write straight into the group's frames
    (rt_render_bands_direct_async, 8-row bands dealt over the S shares).  At world > 1 rank r's
    share j is band rank r*S + j of a world of W*S: its band buffer is slice j of the group's
    [S, B, rows, W, 3] buffer, which is the rank's contribution to ONE gather per group pass
    (rank-major, so the gathered buffer is virtual-rank-major) and rank 0 un-permutes it with
    W*S ranks.

    emulate: rank `rank` of a `world`-rank run on this one GPU with no process group: the same
    slots, groups and passes, every exchange skipped (tools/scale_projection.py)."""

    def __init__(self, scene: DeviceScene, desc, width, height, depth, band_rows=8, rank=0, world=1,
                 device=None, spp=1, seed=0, inflight=4, batch=1, rgb8=False, grid_share=None,
                 force_gather=False, sub_bands=1, emulate=False):
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.inflight = max(1, int(inflight))
        self.world = world
        self.sub_bands = max(1, int(sub_bands))
        S = self.sub_bands
        if S > 1 and (spp != 1 or self.inflight % S):
            raise ValueError("sub_bands > 1: spp 1, inflight a multiple of sub_bands")
        self.groups = self.inflight // S
        self.rank = rank
        self.band_rows = band_rows
        self.w, self.h = width, height
        band_groups = S > 1 and (world > 1 or bool(force_gather))
        self.group_gather = band_groups and not emulate
        scenes = [scene if i == 0 else scene.clone(self.device.index) for i in range(self.inflight)]
        if S == 1:
            self.tilers = [FrameTiler(scenes[i], width, height, depth, band_rows, rank, world, self.device, spp=spp,
                                      seed=seed, batch=batch, rgb8=rgb8, force_gather=force_gather, no_gather=emulate)
                           for i in range(self.inflight)]
        elif not band_groups:
            nb = max(1, min(int(batch), int(abi.lib().rt_max_frames())))
            dt = torch.uint8 if rgb8 else torch.float32
            self.group_frames = [torch.zeros((nb, height, width, 3), dtype=dt, device=self.device)
                                 for _ in range(self.groups)]
            self.tilers = [FrameTiler(scenes[i], width, height, depth, band_rows, i % S, S, self.device, batch=nb,
                                      rgb8=rgb8, frames_out=self.group_frames[i // S])
                           for i in range(self.inflight)]
        else:
            nb = max(1, min(int(batch), int(abi.lib().rt_max_frames())))
            dt = torch.uint8 if rgb8 else torch.float32
            self.vworld = world * S
            rpr = band_rows_per_rank(height, band_rows, self.vworld)
            self.group_local = [torch.zeros((S, nb, rpr, width, 3), dtype=dt, device=self.device)
                                for _ in range(self.groups)]
            self.tilers = [FrameTiler(scenes[i], width, height, depth, band_rows, rank * S + i % S, self.vworld,
                                      self.device, batch=nb, rgb8=rgb8, band_out=self.group_local[i // S][i % S])
                           for i in range(self.inflight)]
            self.group_gathered = self.group_frames = None
            if rank == 0 and self.group_gather:
                self.group_gathered = [torch.zeros((world, S, nb, rpr, width, 3), dtype=dt, device=self.device)
                                       for _ in range(self.groups)]
                self.group_frames = [torch.zeros((nb, height, width, 3), dtype=dt, device=self.device)
                                     for _ in range(self.groups)]
            for i, t in enumerate(self.tilers):
                t.frames = self.group_frames[i // S] if (rank == 0 and self.group_gather) else None
                t.frame = t.frames[0] if t.frames is not None else None
        self.rgb8 = bool(rgb8)
        self.gather = self.tilers[0].gather
        # several passes share the GPU: each pass's persistent trace grids take 75% of the chip
        # (DESIGN.md "Frames in flight"; one pass at a time keeps the whole chip), 50% as band
        # shares -- their passes always run side by side (K = 20, 4 shares, 4 runs each: 35 /
        # 45 / 50 / 55 / 65 / 75%: 1100 / 1121 / 1119 / 1116 / 1108 / 1100 Mpixels/s,
        # profiles/r4ab/)
        self.grid_share = int(grid_share if grid_share is not None else (50 if self.sub_bands > 1 else 75))
        self._caller_share = scene.grid_share   # slot 0 is the caller's scene: restored by close()
        if self.inflight > 1:
            for t in self.tilers:
                t.scene.set_grid_share(self.grid_share)
        self.frame_index = 0        # frames enqueued so far (the `cameras` callback's argument)
        self.pass_index = 0         # passes enqueued so far: pass k runs on group k % groups
        self.batch = self.tilers[0].batch
        self.streams = [torch.cuda.Stream(device=self.device) for _ in range(self.inflight)]
        self._reuse = [None] * self.inflight
        self._whole = None

    @property
    def round_frames(self):
        """frames of one pass on every slot group (the unit of whole passes)"""
        return self.groups * self.batch

    @property
    def counters(self):
        """node rays, shadow rays, pixels summed over the slots"""
        return sum(t.counters for t in self.tilers)

    def zero_counters(self):
        for t in self.tilers:
            t.counters.zero_()

    def group_tilers(self, g):
        return self.tilers[g * self.sub_bands:(g + 1) * self.sub_bands]

    def whole_tiler(self):
        """A tiler of whole frames (batch 1) on slot 0's scene: tilers[0] itself unless the
        slots are band shares (then one made on first use)."""
        if self.sub_bands == 1:
            return self.tilers[0]
        if self._whole is None:
            t0 = self.tilers[0]
            self._whole = FrameTiler(t0.scene, t0.w, t0.h, t0.depth, 8, 0, 1, self.device, rgb8=t0.rgb8)
        return self._whole

    def render_pass(self, g, cams):
        """One pass of group g on the current stream (untimed uses: counting, checks)."""
        for t in self.group_tilers(g):
            t.render_local(len(cams), cams)

    def run(self, n, latency_events=None, cameras=None):
        """Enqueue n frames (asynchronous) in passes of up to `batch` frames, pass k (counted
        across calls) on slot group k % groups; the caller's stream waits for all of them.
        latency_events: a list that receives one (start, end) event pair per pass (per slot).
        cameras: a callable giving the rt_camera of frame i (frames numbered across calls;
        default Camera::new) -- an animation, each frame its own view."""
        main = torch.cuda.current_stream(self.device)
        for s in self.streams:
            s.wait_stream(main)
        while n > 0:
            b = min(self.batch, n)
            n -= b
            g = self.pass_index % self.groups
            self.pass_index += 1
            cams = [cameras(self.frame_index + j) for j in range(b)] if cameras is not None else None
            self.frame_index += b
            for i in range(g * self.sub_bands, (g + 1) * self.sub_bands):
                st = self.streams[i]
                with torch.cuda.stream(st):
                    if self._reuse[i] is not None:
                        st.wait_event(self._reuse[i])
                    if latency_events is not None:
                        ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
                        ev[0].record(st)
                    self.tilers[i].render_local(b, cams)
                    if latency_events is not None:
                        ev[1].record(st)
                        latency_events.append(ev)
                if self.gather:
                    main.wait_stream(st)
                    self.tilers[i].assemble()
                    self._reuse[i] = torch.cuda.Event()
                    self._reuse[i].record(main)
            if self.group_gather:
                self._assemble_group(g, b, main)
        for s in self.streams:
            main.wait_stream(s)

    def _assemble_group(self, g, n, main):
        """One gather of group g's [S, B, rows, W, 3] buffer to rank 0 (on the caller's
        stream, after every share of the pass), then one un-permute of its n frames over the
        W*S virtual ranks; the group's slots wait for it before their next render."""
        S = self.sub_bands
        for i in range(g * S, (g + 1) * S):
            main.wait_stream(self.streams[i])
        local = self.group_local[g]
        world = self.world
        if dist.get_backend() == "gloo":
            host = local.cpu()
            glist = [torch.empty_like(host) for _ in range(world)] if self.rank == 0 else None
            dist.gather(host, gather_list=glist, dst=0)
            if self.rank == 0:
                for r in range(world):
                    self.group_gathered[g][r].copy_(glist[r])
        else:
            glist = [self.group_gathered[g][r] for r in range(world)] if self.rank == 0 else None
            dist.gather(local, gather_list=glist, dst=0)
        if self.rank == 0:
            unpermute_bands_batch_async(self.group_gathered[g].data_ptr(), self.w, self.h, self.band_rows, self.vworld,
                                        n, local.shape[1], self.group_frames[g].data_ptr(),
                                        main.cuda_stream, rgb8=self.rgb8)
        ev = torch.cuda.Event()
        ev.record(main)
        for i in range(g * S, (g + 1) * S):
            self._reuse[i] = ev

    def sync(self):
        """Wait for every slot's enqueued passes; raises RtError(RT_ERR_CAPACITY) if one of
        them overflowed a ray queue (its frames are incomplete -- the slot's next pass gets a
        grown pool, rt_scene_sync_status)."""
        err = None
        for t in self.tilers:  # every slot (each grows its own pool), then the first error
            try:
                t.scene.sync_status()
            except RtError as e:
                err = err or e
        if err is not None:
            raise err

    def _leads(self):
        """one tiler per frame buffer: every slot, or each group's first share"""
        return self.tilers[::self.sub_bands]

    def frames(self):
        """every frame of each slot's (group's) last pass, assembled (rank 0; [] elsewhere).
        Checks every slot's overflow status first: an incomplete frame is never returned."""
        self.sync()
        return [t.frames[b] for t in self._leads() if t.frames is not None for b in range(t.last)]

    def frame_cameras(self):
        """the rt_camera of every frame frames() returns, in the same order"""
        return [t.last_cams[b] for t in self._leads() if t.frames is not None for b in range(t.last)]

    def set_material(self, index, material):
        """rt_scene_set_material on every slot's scene (slot clones are independent copies),
        after the passes enqueued so far (the GUI's material edit, gui.rs:221-236)."""
        torch.cuda.synchronize(self.device)
        for t in self.tilers:
            t.scene.set_material(index, material)

    def close(self):
        for t in self.tilers[1:]:
            t.scene.close()
        self.tilers[0].scene.set_grid_share(self._caller_share)
