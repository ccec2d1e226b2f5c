"""The offline sequence mode (BASELINE config C5) as one object per rank.

`C5Shard` owns everything one rank needs to run the C5 job over its contiguous shard of
the sequence (plus the one-frame halo): the frames rendered on the device into the
batch's level-0 slots, the per-pair buffers, and the step, which runs

  * ORB extraction (C2: ORBextractor(1000, 2.0, 4, 20, 7), ORBextractor.cc:1031-1127),
  * dense Hamming best / second best of frame k against k-1 (ORBmatcher.cc:1507-1523),
  * SparseImgAlign k-1 -> k, levels 3..1 (SparseImageAlign.cc:20-49, Tracking.cc:284),
    map points = frame k-1's keypoints back-projected on the rendered plane,
  * the per-frame result slots packed on the device (ygzfe_batch_pack_slots),
  * with torch.distributed initialised and world > 1, the gather of the slots to rank 0
    (RCCL grouped send / recv over xGMI; `chunks` > 1 gathers chunk c on a communication
    stream while chunk c + 1 computes).

bench.py times `step()`; tests/test_gpu_c5.py runs the same object over the whole
13,728-frame sequence, unsharded and as 8 virtual shards on one GPU, and checks the
slots byte for byte.  `gather=False` keeps a world > 1 shard local (virtual shards).
"""
import numpy as np

from . import dist as D

SWEEP = 240  # frames per sweep of the synthetic trajectory
C5_FRAMES = 3682 + 3040 + 2700 + 2033 + 2273  # EuRoC MH01..MH05 (Examples/Monocular/EuRoC_TimeStamps)
XI = np.array([0.012, -0.006, 0.009, 0.0025, -0.002, 0.0015], np.float32)  # per-frame motion (v, w)
C2 = (752, 480, 1000, 2.0, 4, 20, 7)  # EuRoC.yaml:32-45 (W, H, nFeatures, scale, levels, iniTh, minTh)
SCENE_SEED = 11


def sweep_index(g):
    """Trajectory position of global frame g: 0..SWEEP and back (triangle wave)."""
    k = g % (2 * SWEEP)
    return k if k <= SWEEP else 2 * SWEEP - k


class C5Shard:
    """Rank `rank` of `world` over an `n_seq`-frame C5 sequence on torch device `dev`."""

    def __init__(self, n_seq, rank, world, dev, chunks=1, schedule="serial", align=True, gather=None, scenes=None):
        import torch
        import ygzfe
        if scenes is None:
            from . import scene as scenes  # the textured plane, its constants and pose algebra
        self.S = S = scenes
        self.torch = torch
        self.n_seq, self.rank, self.world, self.dev = n_seq, rank, world, dev
        self.schedule, self.align = schedule, align
        self.schedule_buffers = schedule  # the chunk buffers follow the constructor's schedule
        self.gather = (world > 1) if gather is None else bool(gather)
        W, H, nf, sf, nl, ini, mn = C2
        self.W, self.H = W, H
        self.params = (nf, sf, nl, ini, mn, 0)
        b0, e0 = D.shard(n_seq, rank, world)       # this rank's frames (global indices)
        hb, he = D.with_halo(b0, e0)               # + the halo frame whose pair (b0-1, b0) this rank aligns
        self.b0, self.e0, self.hb, self.he = b0, e0, hb, he
        self.h = h = b0 - hb
        self.F = F = he - hb                       # frames extracted locally
        self.n_own = n_own = e0 - b0
        self.P = P = F - 1                         # align / match pairs (ref p -> cur p+1)
        self.maxlen = -(-n_seq // world)
        self.cam = cam = ygzfe.EUROC_CAM
        self.sc = sc = S.PlaneScene(SCENE_SEED, W, H)
        self.poses = poses = [ygzfe.trajectory_pose(sweep_index(g), XI) for g in range(hb, he)]
        dev_i = dev.index or 0

        self.batch = batch = ygzfe.Batch(self.params, dev_i, W, H, max(F, 2))
        self.cap = cap = batch.kp_cap
        # a real stream shared by torch and ygzfe: torch's default stream is the legacy
        # null stream (handle 0), which ygzfe reads as "the handle's own stream" and which
        # does not order against ygzfe's non-blocking streams
        self.stream = torch.cuda.Stream(dev)
        self.side = torch.cuda.Stream(dev)
        self.sptr = sptr = self.stream.cuda_stream
        self.kps_t = torch.empty((max(F, 2), cap, 7), dtype=torch.float32, device=dev)
        self.counts_t = torch.zeros(max(F, 2), dtype=torch.int32, device=dev)
        self.pyr_t = torch.zeros(max(F, 2) * batch.frame_pitch, dtype=torch.uint8, device=dev)
        batch.bind(pyramids=self.pyr_t.data_ptr(), kps=self.kps_t.data_ptr(), counts=self.counts_t.data_ptr())

        # the sequence rendered on the device straight into the level-0 slots
        with torch.cuda.stream(self.stream):
            tex_d = torch.from_numpy(sc.tex).to(dev)
            q_d = torch.from_numpy(np.stack([q for q, _ in poses])).to(dev)
            t_d = torch.from_numpy(np.stack([t for _, t in poses])).to(dev)
            seeds_d = torch.arange(hb, he, dtype=torch.int64, device=dev)
            ygzfe.render_plane_device(tex_d.data_ptr(), S.TEX_W, S.TEX_H, S.TEXEL, S.PLANE_Z, cam, q_d.data_ptr(),
                                      t_d.data_ptr(), seeds_d.data_ptr(), F, W, H, self.pyr_t.data_ptr(),
                                      batch.frame_pitch, noise_amp=2, stream=sptr)
            self.stream.synchronize()
            del tex_d

            Pp = max(P, 1)
            self.ref_idx = torch.arange(0, Pp, dtype=torch.int32, device=dev)
            self.cur_idx = self.ref_idx + 1
            self.bi = torch.empty((Pp, cap), dtype=torch.int32, device=dev)
            self.bd = torch.empty_like(self.bi)
            self.sd = torch.empty_like(self.bi)
            self.xyz = torch.empty((Pp, cap, 3), dtype=torch.float32, device=dev)
            self.usable = torch.ones((Pp, cap), dtype=torch.uint8, device=dev)
            self.T_init = torch.zeros((Pp, 7), dtype=torch.float32, device=dev)
            self.T_init[:, 3] = 1.0
            self.out = torch.zeros((Pp, 45), dtype=torch.float32, device=dev)
            # plane Z_w = PLANE_Z in each reference camera: X_c = lam * d_c, lam = (Z - C_z) / (r3 . d_c)
            r3 = np.zeros((F, 3), np.float32)
            cz = np.zeros(F, np.float32)
            for i, (q, t) in enumerate(poses):
                qi, ti = S.se3_inv(q.astype(np.float64), t.astype(np.float64))
                R_wc = np.array([S.quat_rot(qi, e) for e in np.eye(3)]).T
                r3[i] = R_wc[2]
                cz[i] = ti[2]
            self.r3, self.cz = r3, cz
            self.r3_t = torch.from_numpy(r3).to(dev)
            self.cz_t = torch.from_numpy(cz).to(dev)
            self.camera = ygzfe.Camera(*cam)
            # result slots: this rank's own frames, padded to the longest shard for the gather
            self.slot_bytes = S_b = ygzfe.slot_bytes(cap)
            self.slots = torch.zeros((self.maxlen, S_b), dtype=torch.uint8, device=dev)
        self.gathered = [torch.empty_like(self.slots) for _ in range(world)] \
            if (self.gather and rank == 0) else None
        self.gather_ms = []

        # ------------------------------------------------ chunked schedule
        # The shard in n_chunks batches bound to consecutive slices of the same device
        # buffers (each with the frame before it, for its first align pair: that frame is
        # extracted twice, identically).  Chunk c's slots are packed into rows [c R, ..)
        # and gathered to rank 0 on `comm` while chunk c + 1 computes on `stream`, so only
        # the last chunk's gather is exposed (ygzfe.dist.chunk_rows / chunk_frames;
        # tests/test_cpu_dist.py checks the layout under gloo).
        self.n_chunks = n_chunks = max(1, chunks)
        self.chunks = []
        self.comm = None
        if n_chunks > 1:
            maxlen_c, Rc = D.chunk_rows(n_seq, world, n_chunks)
            self.slots = torch.zeros((n_chunks * Rc, S_b), dtype=torch.uint8, device=dev)
            self.comm = torch.cuda.Stream(dev)
            # schedule "pipe": two stream pairs, chunks alternating between them
            self.pipe_streams = [(self.stream, self.side), (torch.cuda.Stream(dev), torch.cuda.Stream(dev))]
            # "pipe" runs chunk c + 1's extraction beside chunk c's descriptors and alignment, so
            # the frame they share (chunk c + 1's lead frame) must not be rewritten under chunk
            # c's readers: every chunk gets its own pyramids / rows (level 0 copied once here)
            self.chunk_kps = []
            for c in range(n_chunks):
                s_c, e_c, hc, nc = D.chunk_frames(n_own, h, c, Rc)
                bt = None
                if nc > 0:
                    bt = ygzfe.Batch(self.params, dev_i, W, H, max(e_c - s_c, 2))
                    if schedule == "pipe":
                        Lc = e_c - s_c
                        pyr_c = self.pyr_t[s_c * batch.frame_pitch:e_c * batch.frame_pitch].clone()
                        kps_c = torch.empty((max(Lc, 2), cap, 7), dtype=torch.float32, device=dev)
                        cnt_c = torch.zeros(max(Lc, 2), dtype=torch.int32, device=dev)
                        bt.bind(pyramids=pyr_c.data_ptr(), kps=kps_c.data_ptr(), counts=cnt_c.data_ptr())
                        bt._own = (pyr_c, kps_c, cnt_c)  # kept alive with the batch
                        self.chunk_kps.append(kps_c)
                    else:
                        bt.bind(pyramids=self.pyr_t.data_ptr() + s_c * batch.frame_pitch,
                                kps=self.kps_t[s_c:].data_ptr(), counts=self.counts_t[s_c:].data_ptr())
                        self.chunk_kps.append(self.kps_t[s_c:])
                else:
                    self.chunk_kps.append(None)
                bufs = [torch.empty((Rc, S_b), dtype=torch.uint8, device=dev) for _ in range(world)] \
                    if (rank == 0 and self.gather) else None
                self.chunks.append((s_c, e_c - s_c, hc, nc, bt, bufs, c * Rc))
        self.batches = [ch[4] for ch in self.chunks if ch[4] is not None] if self.chunks else [batch]
        self.F_ext = sum(ch[1] for ch in self.chunks if ch[3] > 0) if self.chunks else F

    # ------------------------------------------------------------------ steps
    def _plane_points(self, off, n, stream=None, kps=None):
        import ygzfe
        kp = self.kps_t[off:] if kps is None else kps
        ygzfe.plane_points_device(kp.data_ptr(), self.cap, n, self.cam, self.r3_t[off:].data_ptr(),
                                  self.cz_t[off:].data_ptr(), self.S.PLANE_Z, self.xyz[off:].data_ptr(),
                                  self.sptr if stream is None else stream)

    def _align(self, bt, off, n, stream=None):
        bt.sparse_align(n, self.ref_idx.data_ptr(), self.cur_idx.data_ptr(), self.xyz[off:].data_ptr(),
                        self.usable[off:].data_ptr(), self.camera, 3, 1, self.T_init[off:].data_ptr(),
                        self.out[off:].data_ptr(), self.sptr if stream is None else stream)

    def _match(self, bt, off, n, stream):
        bt.match(n, self.cur_idx.data_ptr(), self.ref_idx.data_ptr(), self.bi[off:].data_ptr(),
                 self.bd[off:].data_ptr(), self.sd[off:].data_ptr(), stream)

    def _pack_and_gather(self, timed_gather=False):
        import torch.distributed as dist
        torch = self.torch
        P = self.P
        # no align record when align did not run (P == 0 or align off): has_align stays 0
        self.batch.pack_slots(self.h, self.n_own, self.out.data_ptr() if (P > 0 and self.align) else 0, self.b0,
                              self.slots.data_ptr(), self.slot_bytes, self.sptr)
        if self.gather:
            with torch.cuda.stream(self.stream):
                if timed_gather:
                    e0_, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0_.record(self.stream)
                dist.gather(self.slots, self.gathered, dst=0)
                if timed_gather:
                    e1_.record(self.stream)
                    self.gather_ms.append((e0_, e1_))

    def _step_serial(self, timed_gather=False):
        b, P = self.batch, self.P
        b.extract(self.F, self.sptr)
        if P > 0:
            self._match(b, 0, P, self.sptr)
            if self.align:
                self._plane_points(0, P)
                self._align(b, 0, P)
        self._pack_and_gather(timed_gather)

    def _step_tail(self, timed_gather=False):
        # extraction in stage order on `stream` (each extraction kernel has the GPU to
        # itself), then Hamming (descriptors) on `side` beside SparseImgAlign (pyramids +
        # rows) on `stream`
        b, P = self.batch, self.P
        b.extract(self.F, self.sptr)
        self.side.wait_stream(self.stream)
        self._match(b, 0, P, self.side.cuda_stream)
        if self.align:
            self._plane_points(0, P)
            self._align(b, 0, P)
        self.stream.wait_stream(self.side)  # the slots need the match results' descriptors in place
        self._pack_and_gather(timed_gather)

    def _step_split(self, timed_gather=False):
        # keypoint rows on `stream`, blur + descriptors on `side` (the blur runs beside
        # FAST); Hamming (descriptors only) follows on `side`
        b, P = self.batch, self.P
        self.side.wait_stream(self.stream)
        b.extract_split(self.F, self.sptr, self.side.cuda_stream)
        self._match(b, 0, P, self.side.cuda_stream)
        if self.align:
            self._plane_points(0, P)
            if self.schedule == "split":
                # a SparseImgAlign workgroup takes a whole CU: beside orient / Hamming it
                # waits for free CUs and the overlap costs more than it hides
                self.stream.wait_stream(self.side)
            self._align(b, 0, P)
        self.stream.wait_stream(self.side)  # the slots need the descriptors
        self._pack_and_gather(timed_gather)

    def _step_pipe(self, timed_gather=False):
        # software pipeline over the chunks: chunk c on its own stream pair (keypoint rows on
        # `st`, blur + descriptors + Hamming on `sd`, as in the overlap schedule), its start
        # held back until chunk c - 1's keypoint rows are out, so chunk c's pyramid / FAST /
        # octree run beside chunk c - 1's orientation, Hamming and SparseImgAlign
        import torch.distributed as dist
        torch = self.torch
        prev = torch.cuda.Event()
        prev.record(self.stream)  # the previous step's work
        for c, (s_c, L_c, hc, nc, bt, bufs, row0) in enumerate(self.chunks):
            st, sd = self.pipe_streams[c & 1]
            if nc == 0:
                continue
            st.wait_event(prev)
            sd.wait_stream(st)
            Pc = L_c - 1
            bt.extract_split(L_c, st.cuda_stream, sd.cuda_stream)
            prev = torch.cuda.Event()
            prev.record(st)  # chunk c's keypoint rows: the next chunk starts here
            if Pc > 0:
                self._match(bt, s_c, Pc, sd.cuda_stream)
                if self.align:
                    self._plane_points(s_c, Pc, st.cuda_stream, self.chunk_kps[c])
                    self._align(bt, s_c, Pc, st.cuda_stream)
            st.wait_stream(sd)  # the slots need the descriptors
            bt.pack_slots(hc, nc, self.out[s_c:].data_ptr() if (Pc > 0 and self.align) else 0, self.b0 + row0,
                          self.slots[row0:].data_ptr(), self.slot_bytes, st.cuda_stream)
            if self.gather:
                self.comm.wait_stream(st)
                with torch.cuda.stream(self.comm):
                    if timed_gather:
                        e0_, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0_.record(self.comm)
                    dist.gather(self.slots[row0:row0 + (self.slots.shape[0] // self.n_chunks)], bufs, dst=0)
                    if timed_gather:
                        e1_.record(self.comm)
                        self.gather_ms.append((e0_, e1_))
        for st, sd in self.pipe_streams:
            self.stream.wait_stream(st)
            self.stream.wait_stream(sd)
        if self.gather:
            self.stream.wait_stream(self.comm)

    def _step_chunked(self, timed_gather=False):
        import torch.distributed as dist
        torch = self.torch
        for c, (s_c, L_c, hc, nc, bt, bufs, row0) in enumerate(self.chunks):
            if nc > 0:
                Pc = L_c - 1
                bt.extract(L_c, self.sptr)
                if Pc > 0:
                    self._match(bt, s_c, Pc, self.sptr)
                    if self.align:
                        self._plane_points(s_c, Pc, None, self.chunk_kps[c])
                        self._align(bt, s_c, Pc)
                bt.pack_slots(hc, nc, self.out[s_c:].data_ptr() if (Pc > 0 and self.align) else 0, self.b0 + row0,
                              self.slots[row0:].data_ptr(), self.slot_bytes, self.sptr)
            if self.gather:
                ev = torch.cuda.Event()
                ev.record(self.stream)
                self.comm.wait_event(ev)
                with torch.cuda.stream(self.comm):
                    if timed_gather:
                        e0_, e1_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                        e0_.record(self.comm)
                    dist.gather(self.slots[row0:row0 + (self.slots.shape[0] // self.n_chunks)], bufs, dst=0)
                    if timed_gather:
                        e1_.record(self.comm)
                        self.gather_ms.append((e0_, e1_))
        if self.gather:
            self.stream.wait_stream(self.comm)

    def step(self, timed_gather=False):
        if self.chunks and self.schedule == "pipe":
            return self._step_pipe(timed_gather)
        if self.chunks:
            return self._step_chunked(timed_gather)
        if self.schedule == "serial" or self.P == 0:
            return self._step_serial(timed_gather)
        if self.schedule == "tail":
            return self._step_tail(timed_gather)
        return self._step_split(timed_gather)

    # ------------------------------------------------------------------ results
    def counts(self):
        """Keypoints per extracted frame of the shard (F), whichever buffers the schedule used."""
        if self.chunks and self.schedule_buffers == "pipe":
            out = self.torch.zeros(self.F, dtype=self.torch.int32, device=self.dev)
            for (s_c, L_c, hc, nc, bt, bufs, row0) in self.chunks:
                if nc > 0:
                    out[s_c:s_c + L_c] = bt._own[2][:L_c]
            return out
        return self.counts_t[:self.F]

    def check(self):
        for bt in self.batches:
            bt.check()

    def timing(self, enable):
        acc = {}
        for bt in self.batches:
            for k, v in bt.timing(enable).items():
                acc[k] = acc.get(k, 0.0) + v
        return acc

    def local_slots(self):
        """This rank's own frames' slots [n_own, S], in frame order (chunk rows are contiguous)."""
        return self.slots[:self.n_own]

    def root_slots(self):
        """Rank 0 after a gathering step: every frame's slot [n_seq, S] in global order."""
        torch = self.torch
        if not self.gather:
            return self.local_slots() if self.world == 1 else None
        if self.chunks:
            return D.assemble_chunks([ch[5] for ch in self.chunks], self.n_seq, self.world)
        return torch.cat([gg[:D.shard(self.n_seq, r, self.world)[1] - D.shard(self.n_seq, r, self.world)[0]]
                          for r, gg in enumerate(self.gathered)])

    def align_records(self):
        """[P, 45] float32 host copy of the align results (q, t, n_visible, chi2, H)."""
        return self.out[:max(self.P, 1)].cpu().numpy()
