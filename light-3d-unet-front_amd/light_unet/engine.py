"""Forward / backward schedule of Lightweight3DUNet on the gfx950 C-ABI kernels.

Reference semantics: light_unet/models/unet3d.py:146-223 (network), :77-93 (ResidualBlock),
:96-111 (DownBlock), :114-143 (UpBlock).  Every arithmetic op runs in a HIP kernel of
lib/libl3u_hip.so (include/l3u.h); this module only allocates buffers and orders launches on the
current HIP stream, so a whole training step can be captured into one hipGraph.

Memory layout: fp32 NCDHW.  The three decoder concatenations are single buffers
cat_k = [up_k | skip_k]; the encoder block that produces skip_k writes straight into the upper
channel half and the ConvTranspose3d writes the lower half, so torch.cat never copies
(unet3d.py:141).  Their gradients share the same layout.

Partial sums (IN statistics, weight-gradient split-K partials) live in a per-shape arena whose
layout is fixed by a dry run on first use; one l3u_reduce_segments launch at the end of backward
turns all weight-gradient partials into the flat gradient buffer in a fixed order.
"""
import math
import os

import torch

from . import _native as nat

F32 = 4
# the one-input-channel first block's front in one launch (l3u_front_fwd); L3U_FRONT=0 disables
_FRONT = os.environ.get("L3U_FRONT", "1") != "0"
# a block's shortcut and conv1.pointwise GEMMs as one paired launch; L3U_PAIR_PW=0 disables
_PAIR_PW = os.environ.get("L3U_PAIR_PW", "1") != "0"
# outputs per reduction item by partial-list length (<= 128, <= 384, longer); measured best of
# 32..256 on the 48^3 step (tools/seg_caps.sh); L3U_SEG_CAPS overrides
# block-tail backward inside the pointwise backwards (l3u_pw_bwd_tail); L3U_TAIL_FUSE=0 disables
_TAIL_FUSE = os.environ.get("L3U_TAIL_FUSE", "1") != "0"
# (an optional fourth value applies to lists longer than 1024 -- the 48^3 pointwise partials,
# 1728 per layer: round 5 measured 8 outputs per item there +2.6 us on the reduction launch);
# lists of <= 32 partials take 256 outputs per item (fewer workgroups: -3 us, r5p); L3U_SEG_SHORT
# = <max count>:<outputs> overrides
_SEG_CAPS = tuple(int(v) for v in os.environ.get("L3U_SEG_CAPS", "128,64,32").split(","))
_SEG_SHORT = tuple(int(v) for v in os.environ.get("L3U_SEG_SHORT", "32:256").split(":"))
# conv2 (depthwise + pointwise, InstanceNorm1 on load) as one l3u_dwpw_fwd launch for volumes of
# at least this many voxels (the 48^3 level; at 24^3 its 1024-thread slabs are too few to fill
# the chip, tools/dwpw_bench.py); L3U_DWPW=0 disables
_DWPW = os.environ.get("L3U_DWPW", "1") != "0"
# a block's conv2.pointwise and shortcut backwards as one launch at the 12^3 / 6^3 levels
# (l3u_pw_bwd2); L3U_PAIR_BWD=0 keeps them separate
_PAIR_BWD = os.environ.get("L3U_PAIR_BWD", "1") != "0"
# ... and the fused block tail's two pointwise backwards (l3u_pw_bwd_tail_pair) up to this volume
# (48^3: -35 us/step at config 2; at config 5's 64^3 the pair and the accumulating depthwise
# backward cost +100 us, tools/run_evidence.sh step lists) and K ratio (the pair shares one
# column-block width)
_PAIR_TAIL_MAX_S = int(os.environ.get("L3U_PAIR_TAIL_MAX_S", str(48 ** 3)))
# ... and for single-column-block blocks of any channel ratio (the first block's 1 -> 16)
_PAIR_TAIL_NARROW = os.environ.get("L3U_PAIR_TAIL_NARROW", "1") != "0"
_DWPW_MIN_S = int(os.environ.get("L3U_DWPW_MIN_S", "65536"))
# the out_conv backward hands the last block d(pre-sigmoid) and w (out_conv is rank-1) instead
# of the [N, C, S] output gradient (l3u_outconv_bwd_dz + the _r1 tail kernels); L3U_RANK1=0
# disables
_RANK1 = os.environ.get("L3U_RANK1", "1") != "0"
# the encoder's MaxPool3d backward formed in the loads of the consuming block tail (no
# l3u_maxpool2_bwd launch, no level-output gradient tensor); L3U_POOLFOLD=0 disables
_POOLFOLD = os.environ.get("L3U_POOLFOLD", "1") != "0"
# the first block's rank-1 activations (y1 = w1[c] * z1, r = wsc[c] * x: one input channel) are
# never materialised; their consumers form them on load (include/l3u.h "Rank-1 operands", fp32
# only); L3U_FRONT_R1=0 writes them as tensors
_FRONT_R1 = os.environ.get("L3U_FRONT_R1", "1") != "0"
# one process: the backward's final reduction launch also applies the AdamW update of the
# parameters it produces (l3u_reduce_segments_adamw: no separate l3u_adamw_tick launch);
# L3U_FUSE_ADAMW=0 keeps the two launches
_FUSE_ADAMW = os.environ.get("L3U_FUSE_ADAMW", "1") != "0"


# reduction items launched longest first (their workgroups start before the short items fill
# the chip, instead of starting last); L3U_SEG_SORT=0 keeps the recording order
_SEG_SORT = os.environ.get("L3U_SEG_SORT", "1") != "0"


def _seg_rounds(it):
    """Dependent load rounds of one reduction item's threads (misc.hip segment_sum: float4 rows
    when the item allows, 256 // outputs threads per output, 8 loads in flight per thread)."""
    src, cnt, ist, tst, ln, _, _, f64 = it
    vec = not f64 and tst == 1 and ln % 4 == 0 and ist % 4 == 0 and src % 4 == 0
    tp = 256 // (ln // 4) if vec else 256 // ln
    return -(-(-(-cnt // tp)) // 8)


def _items_cover_once(items, numel):
    """True when every one of numel gradient elements is the output of exactly one
    non-accumulating reduction item (the condition of l3u_reduce_segments_adamw)."""
    cnt = torch.zeros(numel, dtype=torch.int32)
    for it in items:
        if it[6]:
            return False
        cnt[it[5]:it[5] + it[4]] += 1
    return bool((cnt == 1).all())


class V:
    """A strided activation view: channel c of sample n at t[off + n*ns + c*S].  scale (a device
    pointer to C floats): a rank-1 tensor, channel c = scale[c] * the one stored channel (a
    gradient: scale passed to the kernel; an activation: the kernel reads the scale from the
    record, `sns` is the batch stride it is given, negative for a rank-1 operand)."""
    __slots__ = ("t", "off", "ns", "C", "scale", "pool")

    def __init__(self, t, off, ns, C, scale=None, pool=None):
        self.t, self.off, self.ns, self.C, self.scale = t, off, ns, C, scale
        # pool = (dpool, idx, (D, H, W)): plus the next level's MaxPool3d backward, formed on load
        self.pool = pool

    @property
    def p(self):
        return self.t.data_ptr() + self.t.element_size() * self.off

    @property
    def sns(self):
        return -self.ns if self.scale is not None else self.ns


def conv_kinds(cin, cout, use_depthwise_separable=True, use_grouped=True, groups=8):
    """(conv1, conv2) of a ResidualBlock as the reference chooses them (unet3d.py:43-60):
    ("ds", 0) DepthwiseSeparableConv3d, ("grouped", G) GroupedConv3d, ("dense", 1) nn.Conv3d."""
    if use_depthwise_separable:
        return ("ds", 0), ("ds", 0)
    k1 = ("grouped", groups) if (use_grouped and groups > 1 and cin >= groups and cout >= groups) \
        else ("dense", 1)
    k2 = ("grouped", groups) if (use_grouped and groups > 1 and cout >= groups) else ("dense", 1)
    return k1, k2


def _conv_params(pre, kind, cin, cout):
    if kind[0] == "ds":
        return [(pre + "depthwise.weight", (cin, 1, 3, 3, 3)),
                (pre + "pointwise.weight", (cout, cin, 1, 1, 1))]
    if kind[0] == "grouped":
        return [(pre + "conv.weight", (cout, cin // kind[1], 3, 3, 3))]
    return [(pre + "weight", (cout, cin, 3, 3, 3))]


def param_layout(enc, in_channels=1, out_channels=1, use_depthwise_separable=True,
                 use_grouped=True, groups=8):
    """(name, shape) in reference registration order (unet3d.py:146-202)."""
    out = []

    def rb(pre, cin, cout, grouped=True):
        k1, k2 = conv_kinds(cin, cout, use_depthwise_separable, use_grouped and grouped, groups)
        out.extend(_conv_params(pre + "conv1.", k1, cin, cout))
        out.extend([(pre + "norm1.weight", (cout,)), (pre + "norm1.bias", (cout,))])
        out.extend(_conv_params(pre + "conv2.", k2, cout, cout))
        out.extend([(pre + "norm2.weight", (cout,)), (pre + "norm2.bias", (cout,))])
        if cin != cout:
            out.extend([(pre + "shortcut.0.weight", (cout, cin, 1, 1, 1)),
                        (pre + "shortcut.1.weight", (cout,)), (pre + "shortcut.1.bias", (cout,))])

    c0, c1, c2, c3 = enc
    rb("init_conv.", in_channels, c0, grouped=False)   # first layer: regular conv (:163-167)
    rb("down1.res_block.", c0, c1)
    rb("down2.res_block.", c1, c2)
    rb("down3.res_block.", c2, c3)
    rb("bottleneck.", c3, c3)
    for name, ci, co in (("up1.", c3, c2), ("up2.", c2, c1), ("up3.", c1, c0)):
        out.append((name + "up.weight", (ci, ci // 2, 2, 2, 2)))
        out.append((name + "up.bias", (ci // 2,)))
        rb(name + "res_block.", ci, co)
    out.append(("out_conv.weight", (out_channels, c0, 1, 1, 1)))
    out.append(("out_conv.bias", (out_channels,)))
    return out


def _splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def stream_seed(base, rank):
    """The Dropout3d seed of data-parallel rank `rank` (rank 0 keeps `base`)."""
    rank = int(rank)
    return int(base) if rank == 0 else _splitmix64((int(base) ^ _splitmix64(rank)) & 0xFFFFFFFFFFFFFFFF)


class _Arena:
    """Bump allocator over one float32 tensor; sized by a dry run on first use of a shape."""

    def __init__(self):
        self.t = None
        self.top = 0

    def reset(self, t):
        self.t, self.top = t, 0

    def alloc(self, n):
        off = self.top
        self.top += (int(n) + 63) & ~63
        return off

    def ptr(self, off):
        return 0 if self.t is None else self.t.data_ptr() + F32 * off


class UNetEngine:
    """Runs Lightweight3DUNet forward/backward on the C-ABI kernels for one architecture."""

    BLOCKS = ("init_conv.", "down1.res_block.", "down2.res_block.", "down3.res_block.",
              "bottleneck.", "up1.res_block.", "up2.res_block.", "up3.res_block.")

    def __init__(self, encoder_channels=(16, 32, 64, 128), in_channels=1, out_channels=1,
                 seed=0x5EED, use_depthwise_separable=True, use_grouped=True, groups=8):
        if in_channels != 1 or out_channels != 1:
            raise NotImplementedError("the MI355X path implements in_channels = out_channels = 1 "
                                      "(the reference's only configuration, trainer.py:57-66)")
        enc = tuple(int(c) for c in encoder_channels)
        if len(enc) != 4 or any(c % 2 for c in enc[1:]):
            raise ValueError(f"encoder_channels must be 4 even ints, got {encoder_channels}")
        if enc[0] > 32:
            raise NotImplementedError("out_conv kernel supports encoder_channels[0] <= 32")
        self.enc = enc
        self.layout = param_layout(enc, use_depthwise_separable=use_depthwise_separable,
                                   use_grouped=use_grouped, groups=groups)
        chans = {"init_conv.": (1, enc[0], False), "down1.res_block.": (enc[0], enc[1], True),
                 "down2.res_block.": (enc[1], enc[2], True), "down3.res_block.": (enc[2], enc[3], True),
                 "bottleneck.": (enc[3], enc[3], True), "up1.res_block.": (enc[3], enc[2], True),
                 "up2.res_block.": (enc[2], enc[1], True), "up3.res_block.": (enc[1], enc[0], True)}
        # per block: the conv kinds of conv1 / conv2 (unet3d.py:43-60)
        self.kinds = {pre: conv_kinds(ci, co, use_depthwise_separable, use_grouped and g, groups)
                      for pre, (ci, co, g) in chans.items()}
        for pre, ks in self.kinds.items():
            for k, (ci, co) in zip(ks, ((chans[pre][0], chans[pre][1]), (chans[pre][1], chans[pre][1]))):
                if k[0] == "grouped" and (ci % k[1] or co % k[1]):
                    raise ValueError(f"{pre}: in_channels {ci} / out_channels {co} must be divisible "
                                     f"by groups {k[1]} (nn.Conv3d)")
        self.offsets = {}
        off = 0
        for name, shape in self.layout:
            n = math.prod(shape)
            self.offsets[name] = (off, n, shape)
            off += n
        self.numel = off
        self.base_seed = int(seed)
        self.stream_id = None   # None: the torch.distributed rank at call time (0 without a group)
        self._arenas = {}
        self._items = {}
        self._cover_once = {}
        self.applied_update = False
        self._dry = False
        self._items_rec = None
        self.seg_bytes = {}    # partial bytes per parameter of the last planned backward
        self.debug = None      # dict -> backward stashes each block's output-gradient view
        self.fwd_arena = _Arena()
        self.bwd_arena = _Arena()
        # activation storage: fp32, or bf16 (BASELINE config 3) through the _bf16 entry points;
        # parameters, records and partial sums stay fp32 either way
        self.act_dtype = torch.float32
        self._grad_phase = False   # backward: gradient buffers are fp32 in either storage mode

    # ------------------------------------------------------------------ helpers
    @property
    def seed(self):
        """Dropout3d stream seed of this process.  The channel-mask hash is (seed, device step,
        layer, n, c) with n the LOCAL sample index, so data-parallel ranks must not share a seed
        (else local sample n draws the same mask on every rank).  Rank 0 (and a single process)
        keeps base_seed, so single-process masks are unchanged; rank r > 0 uses a splitmix of
        (base_seed, r).  stream_id overrides the rank (e.g. a caller-managed stream)."""
        r = self.stream_id
        if r is None:
            import torch.distributed as dist
            r = dist.get_rank() if dist.is_available() and dist.is_initialized() else 0
        return stream_seed(self.base_seed, r)

    def set_act_dtype(self, dtype):
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"activation storage must be float32 or bfloat16, got {dtype}")
        if dtype == torch.bfloat16 and any(k[0][0] != "ds" for k in self.kinds.values()):
            raise NotImplementedError("the bf16 path covers the depthwise-separable network "
                                      "(use_depthwise_separable=True, BASELINE config 3)")
        self.act_dtype = dtype

    @property
    def bf16(self):
        return self.act_dtype == torch.bfloat16

    def _call(self, name, *args):
        """A C-ABI call in the engine's storage mode (the _bf16 twin when activations are bf16)."""
        if not self._dry:
            nat.call(name + "_bf16" if self.bf16 and name in nat.BF16_TWINS else name, *args)

    def _call32(self, name, *args):
        """A call on fp32 operands only (gradient-only GEMMs) in either mode."""
        if not self._dry:
            nat.call(name, *args)

    def _w(self, flat, name):
        return flat.data_ptr() + F32 * self.offsets[name][0]

    def _has(self, name):
        return name in self.offsets

    def _empty(self, *shape, dtype=None, device=None):
        """Forward activations in the engine's storage dtype, backward gradients in fp32, unless
        dtype is given."""
        dt = dtype or (torch.float32 if self._grad_phase else self.act_dtype)
        return torch.empty(shape, dtype=dt, device=device)

    def _f32(self, *shape, device=None):
        return torch.empty(shape, dtype=torch.float32, device=device)

    def _seg(self, src_off, count, istride, tstride, length, dst_name, dst_elem=0, accumulate=0,
             f64=0):
        """Record reduction items: grad[dst_name][dst_elem + t] = sum_i part[src_off+i*is+t*ts].
        f64=1: the partials are fp64 and src_off/strides count doubles from the arena base."""
        base = self.offsets[dst_name][0] + dst_elem
        # outputs per item (one 256-thread workgroup each): fewer for long partial lists so that
        # every thread's serial share stays short (256 / cap threads share each output's terms)
        cap = _SEG_CAPS[0] if count <= 128 else (_SEG_CAPS[1] if count <= 384 else (
            _SEG_CAPS[2] if count <= 1024 or len(_SEG_CAPS) < 4 else _SEG_CAPS[3]))
        if count <= _SEG_SHORT[0]:
            cap = _SEG_SHORT[1]
        t0 = 0
        while t0 < length:
            ln = min(cap, length - t0)
            # misc.hip segment_sum: per-lane offsets from the item's base are 32-bit
            if (count - 1) * istride + (ln - 1) * tstride >= 2 ** 31:
                raise NotImplementedError(f"reduction item for {dst_name} spans more than 2^31 "
                                          "partials from its base (32-bit offsets in segment_sum)")
            self._items_rec.append((src_off + t0 * tstride, count, istride, tstride, ln,
                                    base + t0, accumulate, f64))
            sb = getattr(self, "seg_bytes", None)   # partial bytes per parameter (tools/seg_bytes.py)
            if sb is not None and getattr(self, "_dry", False):
                sb[dst_name] = sb.get(dst_name, 0) + count * ln * (8 if f64 else 4)
            t0 += ln

    @staticmethod
    def check_shape(x):
        if x.dim() != 5 or x.shape[1] != 1:
            raise ValueError(f"expected input [N, 1, D, H, W], got {tuple(x.shape)}")
        _, _, D, H, W = x.shape
        if min(D, H, W) < 8:
            # three MaxPool3d(2) halvings must leave >= 1 voxel (the reference fails there too)
            raise ValueError(f"D, H, W must be >= 8 (three 2x poolings), got {(D, H, W)}")
        for k in range(4):
            h, w = H >> k, W >> k
            # the stencil kernels: x-quad tiles for W % 4 == 0 (W <= 256, any H), whole-plane
            # tiles otherwise (H * W <= 4096)
            if not ((w % 4 == 0 and w <= 256) or h * w <= 4096):
                raise NotImplementedError(
                    f"level-{k} plane {h}x{w}: the stencil kernels need W % 4 == 0 (W <= 256) or "
                    "H * W <= 4096")

    @staticmethod
    def up_pad(lo, hi):
        """UpBlock's F.pad offsets (unet3d.py:130-138): the ConvTranspose3d output 2*lo padded to
        the skip volume hi, diff // 2 before each axis; None when the sizes already match."""
        diff = [h - 2 * l for l, h in zip(lo, hi)]
        if not any(diff):
            return None
        return tuple(d // 2 for d in diff)

    # ------------------------------------------------------------------ forward
    def forward(self, flat, x, training=False, dropout_p=0.0, counter=None, save=True, target=None,
                ftl_part=None, bump_counter=True):
        """x: [N,1,D,H,W] fp32 on device -> probabilities [N,1,D,H,W] (+ saved state).  With a
        target (same shape) the out_conv launch also writes the FocalTversky partials into
        ftl_part [N * l3u_outconv_nblocks(S)][3]."""
        self.check_shape(x)
        x = x.contiguous()
        if x.dtype != torch.float32:
            raise NotImplementedError("the network input is fp32 (bf16 storage is internal)")
        N, _, D, H, W = x.shape
        dev = x.device
        key = ("f", N, D, H, W, self.act_dtype)
        if key not in self._arenas:
            self._dry = True
            self.fwd_arena.reset(None)
            try:
                self._forward_impl(flat, x, training, dropout_p, counter, save, dev, target, ftl_part,
                                   bump_counter)
            finally:
                self._dry = False
            self._arenas[key] = torch.empty(max(self.fwd_arena.top, 64), dtype=torch.float32,
                                            device=dev)
        self.fwd_arena.reset(self._arenas[key])
        return self._forward_impl(flat, x, training, dropout_p, counter, save, dev, target, ftl_part,
                                  bump_counter)

    def _forward_impl(self, flat, x, training, dropout_p, counter, save, dev, target=None,
                      ftl_part=None, bump_counter=True):
        N, _, D, H, W = x.shape
        c0, c1, c2, c3 = self.enc
        dims = [(D >> k, H >> k, W >> k) for k in range(4)]
        S = [d * h * w for d, h, w in dims]
        e = lambda *s: self._empty(*s, device=dev)  # noqa: E731
        drop = dropout_p if training else 0.0
        st = nat.stream()
        sv = {"N": N, "dims": dims, "S": S, "x": x, "drop": drop, "adt": self.act_dtype}
        if drop > 0.0 and counter is not None and bump_counter:
            self._call("l3u_counter_add", counter.data_ptr(), 1, st)
        cptr = counter.data_ptr() if counter is not None else None
        # concatenation buffers [up | skip]
        cat3, cat2, cat1 = e(N, 2 * c0, S[0]), e(N, 2 * c1, S[1]), e(N, 2 * c2, S[2])
        x4 = e(N, c3, S[3])
        sv.update(cat3=cat3, cat2=cat2, cat1=cat1, x4=x4)
        x_in = V(x, 0, S[0], 1)
        if self.bf16 and not self._front_ok(x_in, dims[0]):
            # the bf16 network's input (the front kernel writes this copy itself when it runs)
            xb = e(N, 1, S[0])
            self._call("l3u_cast_f32_bf16", x.data_ptr(), xb.data_ptr(), N * S[0], st)
            x_in = V(xb, 0, S[0], 1)
        x1 = V(cat3, c0 * S[0], 2 * c0 * S[0], c0)
        x2 = V(cat2, c1 * S[1], 2 * c1 * S[1], c1)
        x3 = V(cat1, c2 * S[2], 2 * c2 * S[2], c2)
        x4v = V(x4, 0, c3 * S[3], c3)
        blk = {}
        # the encoder's MaxPool3d inputs x1..x3 and their pooled tensors (DownBlock,
        # unet3d.py:104-105); the pool runs in the producing block's tail when the shape allows
        pools = [(e(N, src.C, S[k + 1]),
                  self._empty(N, src.C, S[k + 1], dtype=torch.uint8, device=dev))
                 for k, src in enumerate((x1, x2, x3))]
        fuse = [self._pool_fusable(src, dims[k]) for k, src in enumerate((x1, x2, x3))]
        blk["init_conv."] = self._block_fwd(flat, "init_conv.", 0, x_in, x1, dims[0], drop, cptr, st,
                                            dev, pool=pools[0] if fuse[0] else None)
        for k, (name, src, dst) in enumerate((("down1.res_block.", x1, x2), ("down2.res_block.", x2, x3),
                                              ("down3.res_block.", x3, x4v))):
            d, h, w = dims[k]
            pooled, idx = pools[k]
            if not fuse[k]:
                self._call("l3u_maxpool2_fwd", src.p, src.ns, pooled.data_ptr(), src.C * S[k + 1],
                           idx.data_ptr(), N, src.C, d, h, w, st)
            pv = V(pooled, 0, src.C * S[k + 1], src.C)
            nxt = pools[k + 1] if k + 1 < 3 and fuse[k + 1] else None
            blk[name] = self._block_fwd(flat, name, k + 1, pv, dst, dims[k + 1], drop, cptr, st, dev,
                                        pool=nxt)
        sv["pools"] = pools
        bott = e(N, c3, S[3])
        blk["bottleneck."] = self._block_fwd(flat, "bottleneck.", 4, x4v, V(bott, 0, c3 * S[3], c3),
                                             dims[3], drop, cptr, st, dev)
        prev = V(bott, 0, c3 * S[3], c3)
        ups = []
        for k, (up, cat, co, lvl) in enumerate((("up1.", cat1, c2, 2), ("up2.", cat2, c1, 1),
                                                ("up3.", cat3, c0, 0))):
            d, h, w = dims[lvl + 1]
            ci = prev.C
            pad = self.up_pad(dims[lvl + 1], dims[lvl])
            if pad is None:   # the scatter epilogue writes the concat buffer's lower half
                self._call("l3u_convt_fwd", prev.p, prev.ns, self._w(flat, up + "up.weight"),
                           self._w(flat, up + "up.bias"), cat.data_ptr(), 2 * co * S[lvl], N, ci,
                           co, d, h, w, st)
            else:             # ragged volume: ConvTranspose3d output, then F.pad into the concat
                upt = e(N, co, 8 * S[lvl + 1])
                self._call("l3u_convt_fwd", prev.p, prev.ns, self._w(flat, up + "up.weight"),
                           self._w(flat, up + "up.bias"), upt.data_ptr(), co * 8 * S[lvl + 1], N,
                           ci, co, d, h, w, st)
                self._call("l3u_box_copy", upt.data_ptr(), co * 8 * S[lvl + 1], 2 * d, 2 * h, 2 * w,
                           cat.data_ptr(), 2 * co * S[lvl], *dims[lvl], *pad, N, co, st)
            out = e(N, co, S[lvl])
            cat_v = V(cat, 0, 2 * co * S[lvl], 2 * co)
            blk[up + "res_block."] = self._block_fwd(flat, up + "res_block.", 5 + k, cat_v,
                                                     V(out, 0, co * S[lvl], co), dims[lvl], drop,
                                                     cptr, st, dev)
            ups.append((prev, out))
            prev = V(out, 0, co * S[lvl], co)
        sv["ups"] = ups
        p = self._f32(N, 1, D, H, W, device=dev)   # probabilities stay fp32 (the loss input)
        # with a target, the FocalTversky first-stage partials come out of the same launch
        self._call("l3u_outconv_fwd", prev.p, prev.ns, self._w(flat, "out_conv.weight"),
                   self._w(flat, "out_conv.bias"), p.data_ptr(),
                   target.data_ptr() if target is not None else None,
                   ftl_part.data_ptr() if target is not None else None, N, c0, S[0], st)
        sv["h"] = prev
        sv["p"] = p
        sv["blk"] = blk
        return p, (sv if save else None)

    def _src(self, flat, norm_prefix, stat_off, nsb, rec_out, drop, cptr, layer, rank1=None):
        """l3u_norm_src for an InstanceNorm whose statistics partials sit at stat_off (rank1: the
        per-channel scale of a rank-1 normalised operand, recorded in the record's slot 7)."""
        return nat.NormSrc(self.fwd_arena.ptr(stat_off), nsb, layer,
                           self._w(flat, norm_prefix + "weight"), self._w(flat, norm_prefix + "bias"),
                           float(drop), self.seed, cptr or 0, rec_out, rank1 or 0)

    @staticmethod
    def _front_ok(x, dims):
        return _FRONT and x.C == 1 and dims[2] % 4 == 0 and x.ns % 4 == 0

    @staticmethod
    def _pool_fusable(v, dims):
        d, h, w = dims
        return d % 2 == 0 and h % 2 == 0 and w % 4 == 0 and v.ns % 4 == 0 and v.p % 16 == 0

    def _block_fwd(self, flat, pre, layer, x, out, dims, drop, cptr, st, dev, pool=None):
        """ResidualBlock.forward (unet3d.py:77-93) into the view `out`; pool = (pooled, idx):
        also the MaxPool3d(2) of the output (the next DownBlock's pool) in the same launch."""
        if self.kinds[pre][0][0] != "ds":
            return self._block_fwd_g(flat, pre, layer, x, out, dims, drop, cptr, st, dev, pool)
        N = x.t.shape[0]
        d, h, w = dims
        S = d * h * w
        cin = x.C
        cout = out.C
        e = lambda *s: self._empty(*s, device=dev)  # noqa: E731
        shortcut = self._has(pre + "shortcut.0.weight")
        nsb = nat.query("l3u_pw_stat_nsb", cin, cout, S)      # pw1 / shortcut (K = cin)
        nsb2 = nat.query("l3u_pw_stat_nsb", cout, cout, S)    # pw2 (K = cout)
        recs = self._f32(3, N * cout, 8, device=dev)
        rec_r, rec1, rec2 = (recs[0].data_ptr(), recs[1].data_ptr(), recs[2].data_ptr())
        sv = {"x": x, "out": out, "recs": recs}
        # InstanceNorm records are finalized inside their consumer kernels from the GEMM
        # partials (l3u_norm_src); `recs` receives them for the backward pass.
        src_r = src2 = None
        if shortcut and self._front_ok(x, dims) and x.t.dtype == torch.float32:
            # the one-input-channel block: shortcut, conv1.depthwise and conv1.pointwise (both
            # rank-1 channel maps) and their IN statistics in one launch (bf16: plus the bf16
            # copy of the input the backward reads)
            nbf = nat.query("l3u_front_nblocks", S)
            r1 = self._front_rank1(x, N, cout, dims)
            z1 = e(N, cin, S)
            r = None if r1 else e(N, cout, S)
            y1 = None if r1 else e(N, cout, S)
            xc = e(N, cin, S) if self.bf16 else None
            so = self.fwd_arena.alloc(N * cout * nbf * 3)
            s1 = self.fwd_arena.alloc(N * cout * nbf * 3)
            self._call("l3u_front_fwd", x.p, x.ns, self._w(flat, pre + "conv1.depthwise.weight"),
                       self._w(flat, pre + "conv1.pointwise.weight"),
                       self._w(flat, pre + "shortcut.0.weight"), z1.data_ptr(),
                       y1.data_ptr() if y1 is not None else None,
                       r.data_ptr() if r is not None else None, self.fwd_arena.ptr(s1),
                       self.fwd_arena.ptr(so), xc.data_ptr() if xc is not None else None, N, cout,
                       d, h, w, st)
            if xc is not None:
                sv["x"] = V(xc, 0, cin * S, cin)
            src_r = self._src(flat, pre + "shortcut.1.", so, nbf, rec_r, 0.0, cptr, 0,
                              rank1=self._w(flat, pre + "shortcut.0.weight") if r1 else None)
            # rank-1: r = wsc[c] * x and y1 = w1[c] * z1 formed on load by every consumer
            rv = V(x.t, x.off, x.ns, cout, scale=self._w(flat, pre + "shortcut.0.weight")) if r1 \
                else V(r, 0, cout * S, cout)
            sv["r"] = rv
            src1 = self._src(flat, pre + "norm1.", s1, nbf, rec1, drop, cptr, 1 + layer,
                             rank1=self._w(flat, pre + "conv1.pointwise.weight") if r1 else None)
        elif _PAIR_PW and shortcut and S % 4 == 0 and x.ns % 4 == 0:
            # conv1.depthwise, then the shortcut and conv1.pointwise (same K -> Nout over the
            # same volume) as one paired GEMM launch
            z1 = e(N, cin, S)
            self._call("l3u_dw3_fwd", x.p, x.ns, self._w(flat, pre + "conv1.depthwise.weight"), None,
                       None, z1.data_ptr(), cin * S, N, cin, d, h, w, st)
            r, y1 = e(N, cout, S), e(N, cout, S)
            so = self.fwd_arena.alloc(N * cout * nsb * 3)
            s1 = self.fwd_arena.alloc(N * cout * nsb * 3)
            self._call("l3u_pw_fwd2", x.p, x.ns, self._w(flat, pre + "shortcut.0.weight"), r.data_ptr(),
                       cout * S, self.fwd_arena.ptr(so), z1.data_ptr(), cin * S,
                       self._w(flat, pre + "conv1.pointwise.weight"), y1.data_ptr(), cout * S,
                       self.fwd_arena.ptr(s1), N, cin, cout, S, st)
            src_r = self._src(flat, pre + "shortcut.1.", so, nsb, rec_r, 0.0, cptr, 0)
            rv = V(r, 0, cout * S, cout)
            sv["r"] = rv
            src1 = self._src(flat, pre + "norm1.", s1, nsb, rec1, drop, cptr, 1 + layer)
        else:
            if shortcut:
                r = e(N, cout, S)
                so = self.fwd_arena.alloc(N * cout * nsb * 3)
                self._call("l3u_pw_fwd", x.p, x.ns, self._w(flat, pre + "shortcut.0.weight"), 0,
                           None, r.data_ptr(), cout * S, 0, self.fwd_arena.ptr(so), N, cin, cout, S,
                           st)
                src_r = self._src(flat, pre + "shortcut.1.", so, nsb, rec_r, 0.0, cptr, 0)
                rv = V(r, 0, cout * S, cout)
                sv["r"] = rv
            else:
                rv = x
                sv["r"] = None
            z1 = e(N, cin, S)
            self._call("l3u_dw3_fwd", x.p, x.ns, self._w(flat, pre + "conv1.depthwise.weight"), None,
                       None, z1.data_ptr(), cin * S, N, cin, d, h, w, st)
            y1 = e(N, cout, S)
            s1 = self.fwd_arena.alloc(N * cout * nsb * 3)
            self._call("l3u_pw_fwd", z1.data_ptr(), cin * S,
                       self._w(flat, pre + "conv1.pointwise.weight"), 0, None, y1.data_ptr(),
                       cout * S, 0, self.fwd_arena.ptr(s1), N, cin, cout, S, st)
            src1 = self._src(flat, pre + "norm1.", s1, nsb, rec1, drop, cptr, 1 + layer)
        z2 = e(N, cout, S)
        y2 = e(N, cout, S)
        # y1 as conv2 reads it: a tensor, or rank-1 (z1 with a negative batch stride)
        y1v = V(z1, 0, S, cout, scale=True) if y1 is None else V(y1, 0, cout * S, cout)
        if self._use_dwpw(cout, dims):
            # conv2 = depthwise (IN1 + LeakyReLU + Dropout3d on load) + pointwise in one launch
            nsb2 = nat.query("l3u_dwpw_stat_nsb", cout, cout, d, h, w)
            s2 = self.fwd_arena.alloc(N * cout * nsb2 * 3)
            self._call("l3u_dwpw_fwd", y1v.p, y1v.sns,
                       self._w(flat, pre + "conv2.depthwise.weight"), None, nat.norm_src_ptr(src1),
                       self._w(flat, pre + "conv2.pointwise.weight"), y2.data_ptr(), cout * S,
                       self.fwd_arena.ptr(s2), None, None, 0, None, z2.data_ptr(), cout * S, N, cout,
                       cout, d, h, w, st)
        else:
            # (a rank-1 y1 goes in with its negative batch stride: l3u_dw3_fwd forms w1[c] * z1
            # on load, l3u_dw3_bwd_rank1 shapes)
            self._call("l3u_dw3_fwd", y1v.p, y1v.sns,
                       self._w(flat, pre + "conv2.depthwise.weight"), None, nat.norm_src_ptr(src1),
                       z2.data_ptr(), cout * S, N, cout, d, h, w, st)
            s2 = self.fwd_arena.alloc(N * cout * nsb2 * 3)
            self._call("l3u_pw_fwd", z2.data_ptr(), cout * S,
                       self._w(flat, pre + "conv2.pointwise.weight"), 0, None, y2.data_ptr(), cout * S,
                       0, self.fwd_arena.ptr(s2), N, cout, cout, S, st)
        src2 = self._src(flat, pre + "norm2.", s2, nsb2, rec2, 0.0, cptr, 0)
        if pool is None:
            self._call("l3u_norm_act_fwd", y2.data_ptr(), cout * S, None, nat.norm_src_ptr(src2),
                       rv.p, rv.sns, None, nat.norm_src_ptr(src_r), 1 if shortcut else 0, out.p,
                       out.ns, N, cout, S, st)
        else:
            pooled, idx = pool
            self._call("l3u_norm_act_pool_fwd", y2.data_ptr(), cout * S, None,
                       nat.norm_src_ptr(src2), rv.p, rv.sns, None, nat.norm_src_ptr(src_r),
                       1 if shortcut else 0, out.p, out.ns, pooled.data_ptr(), cout * (S // 8),
                       idx.data_ptr(), N, cout, d, h, w, st)
        sv.update(z1=z1, y1=y1, y1v=y1v, z2=z2, y2=y2, dims=dims, shortcut=shortcut)
        return sv

    @staticmethod
    def _use_dwpw(cout, dims):
        """conv2 as the one-launch l3u_dwpw_fwd (else l3u_dw3_fwd then l3u_pw_fwd)."""
        d, h, w = dims
        return (_DWPW and d * h * w >= _DWPW_MIN_S
                and nat.query("l3u_dwpw_supported", cout, cout, d, h, w, 0) == 1)

    def _front_rank1(self, x, N, cout, dims):
        """The first block's y1 / r stay rank-1 (never materialised) when every consumer takes a
        rank-1 operand at this shape: the fused conv2 (l3u_dwpw_fwd), the LDS-DMA IN-fused
        depthwise backward, the fused pointwise backwards and the fused block tail (fp32)."""
        d, h, w = dims
        S = d * h * w
        return (_FRONT_R1 and not self.bf16 and self._front_ok(x, dims)
                # conv2's forward takes the rank-1 y1 (the fused l3u_dwpw_fwd, or l3u_dw3_fwd) at
                # the l3u_dw3_bwd_rank1 shapes, as the IN-fused depthwise backward does
                and nat.query("l3u_dw3_bwd_rank1", N, cout, d, h, w)
                and nat.query("l3u_pw_bwd_supported", cout, 1, S)
                # the rank-1 pointwise backward variants take one 16-column block (J = cout <= 16)
                and _TAIL_FUSE and nat.query("l3u_norm_act_nblocks", S) > 1 and cout <= 16
                and nat.query("l3u_pw_bwd_supported", cout, cout, S))

    def _conv_w(self, flat, pre, which):
        kind = self.kinds[pre][which - 1]
        name = pre + f"conv{which}." + ("conv.weight" if kind[0] == "grouped" else "weight")
        return name, self._w(flat, name), (kind[1] if kind[0] == "grouped" else 1)

    def _block_fwd_g(self, flat, pre, layer, x, out, dims, drop, cptr, st, dev, pool=None):
        """ResidualBlock.forward with grouped / dense 3^3 convs (use_depthwise_separable=False,
        unet3d.py:43-60,77-93): conv1 -> IN1 (record finalized from the conv's statistics
        partials) -> conv2 with IN1 + LeakyReLU + Dropout3d applied on its input load -> the
        same fused block tail as the depthwise-separable path."""
        N = x.t.shape[0]
        d, h, w = dims
        S = d * h * w
        cin, cout = x.C, out.C
        e = lambda *s: self._empty(*s, device=dev)  # noqa: E731
        nsb = nat.query("l3u_pw_stat_nsb", cin, cout, S)
        nbg = nat.query("l3u_gconv3_nblocks", S)
        recs = self._f32(3, N * cout, 8, device=dev)
        rec_r, rec1, rec2 = (recs[0].data_ptr(), recs[1].data_ptr(), recs[2].data_ptr())
        sv = {"x": x, "out": out, "recs": recs}
        shortcut = self._has(pre + "shortcut.0.weight")
        src_r = None
        if shortcut:
            r = e(N, cout, S)
            so = self.fwd_arena.alloc(N * cout * nsb * 3)
            self._call("l3u_pw_fwd", x.p, x.ns, self._w(flat, pre + "shortcut.0.weight"), 0, None,
                       r.data_ptr(), cout * S, 0, self.fwd_arena.ptr(so), N, cin, cout, S, st)
            src_r = self._src(flat, pre + "shortcut.1.", so, nsb, rec_r, 0.0, cptr, 0)
            rv = V(r, 0, cout * S, cout)
            sv["r"] = rv
        else:
            rv = x
            sv["r"] = None
        _, w1, g1 = self._conv_w(flat, pre, 1)
        _, w2, g2 = self._conv_w(flat, pre, 2)
        y1 = e(N, cout, S)
        s1 = self.fwd_arena.alloc(N * cout * nbg * 3)
        self._call("l3u_gconv3_fwd", x.p, x.ns, w1, None, y1.data_ptr(), cout * S,
                   self.fwd_arena.ptr(s1), N, cin, cout, g1, d, h, w, st)
        self._call("l3u_in_finalize", self.fwd_arena.ptr(s1), nbg, self._w(flat, pre + "norm1.weight"),
                   self._w(flat, pre + "norm1.bias"), float(drop), self.seed, cptr, 1 + layer, rec1,
                   N, cout, st)
        y2 = e(N, cout, S)
        s2 = self.fwd_arena.alloc(N * cout * nbg * 3)
        self._call("l3u_gconv3_fwd", y1.data_ptr(), cout * S, w2, rec1, y2.data_ptr(), cout * S,
                   self.fwd_arena.ptr(s2), N, cout, cout, g2, d, h, w, st)
        src2 = self._src(flat, pre + "norm2.", s2, nbg, rec2, 0.0, cptr, 0)
        if pool is None:
            self._call("l3u_norm_act_fwd", y2.data_ptr(), cout * S, None, nat.norm_src_ptr(src2),
                       rv.p, rv.ns, None, nat.norm_src_ptr(src_r), 1 if shortcut else 0, out.p,
                       out.ns, N, cout, S, st)
        else:
            pooled, idx = pool
            self._call("l3u_norm_act_pool_fwd", y2.data_ptr(), cout * S, None,
                       nat.norm_src_ptr(src2), rv.p, rv.ns, None, nat.norm_src_ptr(src_r),
                       1 if shortcut else 0, out.p, out.ns, pooled.data_ptr(), cout * (S // 8),
                       idx.data_ptr(), N, cout, d, h, w, st)
        sv.update(y1=y1, y2=y2, dims=dims, shortcut=shortcut)
        return sv

    # ------------------------------------------------------------------ backward
    def backward(self, flat, gflat, sv, dp, need_dx=False, ftl=None, opt=None):
        """Given dL/dp write all parameter gradients into gflat (overwrite) and return dL/dx if
        need_dx.  opt: the FlatAdamW over (flat, gflat) of a one-process step; when the gradient
        reduction covers every parameter once, its launch also applies the update and
        self.applied_update is True (the caller must then not call opt.step()).  dp = None: the loss is FocalTversky and ftl = (target, global sums [3] fp64,
        (alpha, beta, gamma, smooth)[, loss tensor[, partials, n_partials]]); its gradient is
        formed inside the out_conv backward, which also writes the loss value when a loss tensor
        is given.  sums = None: the out_conv backward reduces the forward's FocalTversky
        partials itself (l3u_outconv_bwd_ftl; no reduce launch)."""
        N = sv["N"]
        D, H, W = sv["dims"][0]
        self.set_act_dtype(sv["adt"])
        key = ("b", N, D, H, W, bool(need_dx), self.act_dtype)
        self._grad_phase = True
        try:
            if key not in self._arenas:
                self._dry = True
                self.bwd_arena.reset(None)
                self._items_rec = []
                self.seg_bytes = {}
                try:
                    self._backward_impl(flat, gflat, sv, dp, need_dx, ftl)
                finally:
                    self._dry = False
                dev = sv["p"].device
                self._arenas[key] = torch.empty(max(self.bwd_arena.top, 64), dtype=torch.float32,
                                                device=dev)
                # items are independent (each output is written by one item), so their order
                # changes no result
                rec = sorted(self._items_rec, key=lambda it: -_seg_rounds(it)) if _SEG_SORT \
                    else self._items_rec
                self._items[key] = torch.tensor(rec, dtype=torch.int64, device=dev)
                self._cover_once[key] = _items_cover_once(self._items_rec, gflat.numel())
            self.bwd_arena.reset(self._arenas[key])
            self._items_rec = []
            dx = self._backward_impl(flat, gflat, sv, dp, need_dx, ftl)
        finally:
            self._grad_phase = False
        items = self._items[key]
        self.applied_update = (opt is not None and _FUSE_ADAMW and self._cover_once[key]
                               and opt.g is gflat and opt.p is flat)
        if self.applied_update:
            nat.call("l3u_reduce_segments_adamw", self.bwd_arena.ptr(0), items.data_ptr(),
                     items.shape[0], *opt.fused_args(), nat.stream())
        else:
            nat.call("l3u_reduce_segments", self.bwd_arena.ptr(0), items.data_ptr(),
                     items.shape[0], gflat.data_ptr(), nat.stream())
        return dx

    def _backward_impl(self, flat, gflat, sv, dp, need_dx, ftl=None):
        N = sv["N"]
        dims, S = sv["dims"], sv["S"]
        c0, c1, c2, c3 = self.enc
        dev = sv["p"].device
        e = lambda *s: self._empty(*s, device=dev)  # noqa: E731
        st = nat.stream()
        A = self.bwd_arena
        # ---- out_conv + sigmoid (unet3d.py:220-221)
        h = sv["h"]
        up3 = sv["blk"]["up3.res_block."]
        # rank-1 hand-off: the tail kernels of the last block form dout[c] = w[c] * dz themselves
        r1 = _RANK1 and self.kinds["up3.res_block."][0][0] == "ds" and \
            self._tail_fusable(up3, up3["x"].C, c0, S[0])
        sfx = "_dz" if r1 else ""
        dh = e(N, 1, S[0]) if r1 else e(N, c0, S[0])
        dhns = S[0] if r1 else c0 * S[0]
        nb = nat.query("l3u_outconv_nblocks", S[0])
        po = A.alloc(2 * N * nb * (c0 + 1))          # fp64 partials
        loss_ptr = None
        if dp is not None:
            g = (dp.data_ptr(), None, None, 0.0, 0.0, 0.0, 0.0, None)
            self._call("l3u_outconv_bwd" + sfx, g[0], sv["p"].data_ptr(), *g[1:], h.p, h.ns,
                       self._w(flat, "out_conv.weight"), dh.data_ptr(), dhns, A.ptr(po),
                       loss_ptr, N, c0, S[0], st)
        else:   # FocalTversky gradient formed inside the kernel from the global sums
            t, sums, (alpha, beta, gamma, smooth) = ftl[:3]
            if len(ftl) > 3 and ftl[3] is not None:   # the loss value, written by the same launch
                loss_ptr = ftl[3].data_ptr()
            if sums is None:   # the sums reduced inside the launch from the forward's partials
                fpart, fnp = ftl[4], ftl[5]
                self._call("l3u_outconv_bwd_ftl" + sfx, sv["p"].data_ptr(), t.data_ptr(),
                           fpart.data_ptr(), fnp, alpha, beta, gamma, smooth, None, h.p, h.ns,
                           self._w(flat, "out_conv.weight"), dh.data_ptr(), dhns, A.ptr(po),
                           loss_ptr, N, c0, S[0], st)
            else:
                self._call("l3u_outconv_bwd" + sfx, None, sv["p"].data_ptr(), t.data_ptr(),
                           sums.data_ptr(), alpha, beta, gamma, smooth, None, h.p, h.ns,
                           self._w(flat, "out_conv.weight"), dh.data_ptr(), dhns, A.ptr(po),
                           loss_ptr, N, c0, S[0], st)
        self._seg(po // 2, N * nb, c0 + 1, 1, c0, "out_conv.weight", f64=1)
        self._seg(po // 2 + c0, N * nb, c0 + 1, 1, 1, "out_conv.bias", f64=1)
        dcat3, dcat2, dcat1 = e(N, 2 * c0, S[0]), e(N, 2 * c1, S[1]), e(N, 2 * c2, S[2])
        dcats = {0: dcat3, 1: dcat2, 2: dcat1}
        dout = V(dh, 0, dhns, c0, self._w(flat, "out_conv.weight") if r1 else None)
        # ---- decoder (reverse order); up_specs = (prefix, Co, level, index into sv["ups"])
        up_specs = [("up3.", c0, 0, 2), ("up2.", c1, 1, 1), ("up1.", c2, 2, 0)]
        for up, co, lvl, uidx in up_specs:
            dcat = dcats[lvl]
            self._block_bwd(flat, up + "res_block.", sv["blk"][up + "res_block."], dout,
                            V(dcat, 0, 2 * co * S[lvl], 2 * co), st, dev)
            # ConvTranspose3d backward: input = prev (the lower-level output), dOut = dcat[:, :co]
            prev, _ = sv["ups"][uidx]
            ci = prev.C
            d, hh, w = dims[lvl + 1]
            dprev = e(N, ci, S[lvl + 1])
            # dY read in place from the lower half of the concat gradient (ragged volume: cropped
            # to the ConvTranspose3d output first, the backward of F.pad)
            dY, dYns = dcat.data_ptr(), 2 * co * S[lvl]
            pad = self.up_pad(dims[lvl + 1], dims[lvl])
            if pad is not None:
                dup = self._f32(N, co, 8 * S[lvl + 1], device=dev)
                self._call32("l3u_box_copy", dY, dYns, *dims[lvl], dup.data_ptr(), co * 8 * S[lvl + 1],
                             2 * d, 2 * hh, 2 * w, *[-o for o in pad], N, co, st)
                dY, dYns = dup.data_ptr(), co * 8 * S[lvl + 1]
            npf = nat.query("l3u_convt_bwd_fused_nparts", N, ci, co, d, hh, w)
            if npf > 0:   # one launch: data, weight and bias gradients
                pw, pb = A.alloc(npf * ci * co * 8), A.alloc(npf * co)
                self._call("l3u_convt_bwd_fused", dY, dYns, prev.p, prev.ns,
                           self._w(flat, up + "up.weight"), dprev.data_ptr(), ci * S[lvl + 1],
                           A.ptr(pw), A.ptr(pb), N, ci, co, d, hh, w, st)
                self._seg(pw, npf, ci * co * 8, 1, ci * co * 8, up + "up.weight")
                self._seg(pb, npf, co, 1, co, up + "up.bias")
            else:
                npw = nat.query("l3u_pw_bwd_weight_nparts", N, S[lvl + 1])
                pw, pb = A.alloc(npw * ci * co * 8), A.alloc(npw * co)
                self._call("l3u_convt_bwd", dY, dYns, prev.p, prev.ns,
                           self._w(flat, up + "up.weight"), dprev.data_ptr(), ci * S[lvl + 1],
                           A.ptr(pw), A.ptr(pb), N, ci, co, d, hh, w, st)
                self._seg(pw, npw, ci * co * 8, 1, ci * co * 8, up + "up.weight")
                self._seg(pb, npw, co, 1, co, up + "up.bias")
            dout = V(dprev, 0, ci * S[lvl + 1], ci)
        # ---- bottleneck
        dx4 = e(N, c3, S[3])
        self._block_bwd(flat, "bottleneck.", sv["blk"]["bottleneck."], dout,
                        V(dx4, 0, c3 * S[3], c3), st, dev)
        dout = V(dx4, 0, c3 * S[3], c3)
        # ---- encoder
        enc_specs = [("down3.res_block.", c2, 2), ("down2.res_block.", c1, 1),
                     ("down1.res_block.", c0, 0)]
        for name, cprev, lvl in enc_specs:
            pooled, idx = sv["pools"][lvl]
            dpool = e(N, cprev, S[lvl + 1])
            self._block_bwd(flat, name, sv["blk"][name], dout, V(dpool, 0, cprev * S[lvl + 1], cprev),
                            st, dev)
            # d(level output) = maxpool_bwd(dpool) + d(skip) (upper half of dcat at this level)
            dcat = dcats[lvl]
            d, hh, w = dims[lvl]
            cons = ("init_conv.", "down1.res_block.", "down2.res_block.")[lvl]
            csv = sv["blk"][cons]
            if (_POOLFOLD and self.kinds[cons][0][0] == "ds" and d % 2 == 0 and hh % 2 == 0
                    and w % 4 == 0 and (self._tail_fusable(csv, csv["x"].C, cprev, S[lvl])
                                        or self._tail_one_up(csv, S[lvl]))):
                # the consuming block tail forms it on load (l3u_*_up): no tensor, no launch
                dout = V(dcat, cprev * S[lvl], 2 * cprev * S[lvl], cprev, pool=(dpool, idx, dims[lvl]))
                continue
            dlev = e(N, cprev, S[lvl])
            self._call("l3u_maxpool2_bwd", dpool.data_ptr(), cprev * S[lvl + 1], idx.data_ptr(),
                       dcat.data_ptr() + dcat.element_size() * cprev * S[lvl], 2 * cprev * S[lvl],
                       dlev.data_ptr(),
                       cprev * S[lvl], N, cprev, d, hh, w, st)
            dout = V(dlev, 0, cprev * S[lvl], cprev)
        # ---- init block
        dx = e(N, 1, *dims[0])
        self._block_bwd(flat, "init_conv.", sv["blk"]["init_conv."], dout, V(dx, 0, S[0], 1),
                        st, dev)
        return dx if need_dx else None

    def _tail_fusable(self, sv, cin, cout, S):
        """The block tail's backward can ride in the prologues of the two pointwise backwards
        (l3u_pw_bwd_tail) instead of l3u_norm_act_bwd_apply: Conv1x1 shortcut, several
        workgroups per plane (one-workgroup planes take the one-launch l3u_norm_act_bwd) and
        the fused-kernel shapes for conv2.pointwise (J = K = cout) and the shortcut (K = cin)."""
        return (_TAIL_FUSE and sv["shortcut"] and nat.query("l3u_norm_act_nblocks", S) > 1
                and cout <= 32 and nat.query("l3u_pw_bwd_supported", cout, cout, S)
                and nat.query("l3u_pw_bwd_supported", cout, cin, S))

    @staticmethod
    def _tail_one_up(sv, S):
        """An unfused block tail whose planes take the one-launch l3u_norm_act_bwd can form its
        output gradient on load as well (l3u_norm_act_bwd_up, the register-held planes <= 2048
        voxels: the 12^3 level), without a rank-1 residual."""
        return (nat.query("l3u_norm_act_nblocks", S) == 1 and S <= 2048
                and (sv["r"] if sv["shortcut"] else sv["x"]).scale is None)

    def _tail_bwd(self, pre, sv, dout, dxv, N, cout, S, st, dev, fused=False):
        """Backward of the block tail out = lrelu(IN2(y2) + residual): d y2 and d residual (the
        shortcut-conv output, or dxv itself for the identity shortcut), with the norm2 / shortcut
        IN parameter-gradient reductions recorded.  fused: only the reduce; returns the tail
        partials' arena offset for l3u_pw_bwd_tail instead."""
        A = self.bwd_arena
        out, recs = sv["out"], sv["recs"]
        rec_r, rec2 = recs[0].data_ptr(), recs[2].data_ptr()
        shortcut = sv["shortcut"]
        rv = sv["r"] if shortcut else sv["x"]
        y2 = sv["y2"]
        nb = nat.query("l3u_norm_act_nblocks", S)
        pn = A.alloc(2 * cout * N * nb * 3)            # fp64 partials
        pnd = pn // 2
        self._seg(pnd + 1, N * nb, 3, N * nb * 3, cout, pre + "norm2.weight", f64=1)
        self._seg(pnd + 0, N * nb, 3, N * nb * 3, cout, pre + "norm2.bias", f64=1)
        if fused:
            self._seg(pnd + 2, N * nb, 3, N * nb * 3, cout, pre + "shortcut.1.weight", f64=1)
            self._seg(pnd + 0, N * nb, 3, N * nb * 3, cout, pre + "shortcut.1.bias", f64=1)
            if dout.scale is not None:   # rank-1 dout (l3u_outconv_bwd_dz)
                self._call("l3u_norm_act_bwd_reduce_r1", dout.p, dout.ns, dout.scale, out.p, out.ns,
                           y2.data_ptr(), cout * S, rec2, rv.p, rv.sns, rec_r, A.ptr(pn), N, cout, S,
                           st)
            elif dout.pool is not None:   # skip gradient + the folded MaxPool3d backward
                dpool, idx, (d, h, w) = dout.pool
                self._call("l3u_norm_act_bwd_reduce_up", dout.p, dout.ns, dpool.data_ptr(),
                           cout * (S // 8), idx.data_ptr(), out.p, out.ns, y2.data_ptr(), cout * S,
                           rec2, rv.p, rv.sns, rec_r, A.ptr(pn), N, cout, d, h, w, st)
            else:
                self._call("l3u_norm_act_bwd_reduce", dout.p, dout.ns, out.p, out.ns, y2.data_ptr(),
                           cout * S, rec2, rv.p, rv.sns, rec_r, A.ptr(pn), N, cout, S, st)
            return pn, nb
        assert dout.scale is None and (dout.pool is None or nb == 1), "a formed-on-load output " \
            "gradient needs the fused block tail or a one-launch plane"
        assert rv.scale is None, "a rank-1 residual needs the fused block tail"
        dy2 = self._empty(N, cout, S, device=dev)
        if shortcut:
            dr = self._empty(N, cout, S, device=dev)
            drv = V(dr, 0, cout * S, cout)
            self._seg(pnd + 2, N * nb, 3, N * nb * 3, cout, pre + "shortcut.1.weight", f64=1)
            self._seg(pnd + 0, N * nb, 3, N * nb * 3, cout, pre + "shortcut.1.bias", f64=1)
        else:
            drv = dxv   # identity shortcut: d(input) starts as g
        if nb == 1 and dout.pool is not None:   # + the folded MaxPool3d backward
            dpool, idx, (d, h, w) = dout.pool
            self._call("l3u_norm_act_bwd_up", dout.p, dout.ns, dpool.data_ptr(), cout * (S // 8),
                       idx.data_ptr(), out.p, out.ns, y2.data_ptr(), cout * S, rec2, rv.p, rv.ns,
                       rec_r if shortcut else None, A.ptr(pn), dy2.data_ptr(), cout * S, drv.p,
                       drv.ns, N, cout, d, h, w, st)
            return dy2, drv
        if nb == 1:   # one workgroup per plane: reduce and apply in one launch
            self._call("l3u_norm_act_bwd", dout.p, dout.ns, out.p, out.ns, y2.data_ptr(), cout * S,
                       rec2, rv.p, rv.ns, rec_r if shortcut else None, A.ptr(pn), dy2.data_ptr(),
                       cout * S, drv.p, drv.ns, N, cout, S, st)
            return dy2, drv
        self._call("l3u_norm_act_bwd_reduce", dout.p, dout.ns, out.p, out.ns, y2.data_ptr(), cout * S,
                   rec2, rv.p, rv.ns, rec_r if shortcut else None, A.ptr(pn), N, cout, S, st)
        self._call("l3u_norm_act_bwd_apply", dout.p, dout.ns, out.p, out.ns, y2.data_ptr(), cout * S,
                   rec2, rv.p, rv.ns, rec_r if shortcut else None, A.ptr(pn), dy2.data_ptr(),
                   cout * S, drv.p, drv.ns, N, cout, S, st)
        return dy2, drv

    def _block_bwd_g(self, flat, pre, sv, dout, dxv, st, dev):
        """Backward of the grouped / dense ResidualBlock (_block_fwd_g)."""
        A = self.bwd_arena
        x, recs = sv["x"], sv["recs"]
        if self.debug is not None and not self._dry:
            self.debug[pre] = dout
        d, h, w = sv["dims"]
        S = d * h * w
        N = x.t.shape[0]
        cin, cout = x.C, sv["out"].C
        rec1 = recs[1].data_ptr()
        shortcut = sv["shortcut"]
        y1 = sv["y1"]
        dy2, drv = self._tail_bwd(pre, sv, dout, dxv, N, cout, S, st, dev)
        n1, w1, g1 = self._conv_w(flat, pre, 1)
        n2, w2, g2 = self._conv_w(flat, pre, 2)
        nbg = nat.query("l3u_gconv3_nblocks", S)
        P = nat.query("l3u_gconv3_wgrad_nparts", N, S)
        # conv2: data gradient with the LeakyReLU/Dropout/IN1 backward partials, weight gradient
        # against the IN1-transformed input (recomputed from y1)
        pi1 = A.alloc(2 * cout * N * nbg * 2)          # fp64 partials
        pid = pi1 // 2
        dpre = self._empty(N, cout, S, device=dev)
        self._call("l3u_gconv3_bwd_data", dy2.data_ptr(), cout * S, w2, rec1, y1.data_ptr(), cout * S,
                   dpre.data_ptr(), cout * S, 0, A.ptr(pi1), N, cout, cout, g2, d, h, w, st)
        pw2 = A.alloc(P * cout * (cout // g2) * 27)
        self._call("l3u_gconv3_bwd_weight", dy2.data_ptr(), cout * S, y1.data_ptr(), cout * S, rec1,
                   A.ptr(pw2), N, cout, cout, g2, d, h, w, st)
        n2w = cout * (cout // g2) * 27
        self._seg(pw2, P, n2w, 1, n2w, n2)
        self._seg(pid + 1, N * nbg, 2, N * nbg * 2, cout, pre + "norm1.weight", f64=1)
        self._seg(pid + 0, N * nbg, 2, N * nbg * 2, cout, pre + "norm1.bias", f64=1)
        # IN1 backward: dy1 = IN-backward(dpre) in place
        self._call("l3u_in_bwd_apply", dpre.data_ptr(), cout * S, y1.data_ptr(), cout * S, rec1,
                   A.ptr(pi1), nbg, dpre.data_ptr(), cout * S, N, cout, S, st)
        dy1 = dpre
        # conv1: d(input) (overwrite for the Conv1x1 shortcut, accumulate onto the identity
        # shortcut's gradient) and the weight gradient
        self._call("l3u_gconv3_bwd_data", dy1.data_ptr(), cout * S, w1, None, None, 0, dxv.p, dxv.ns,
                   0 if shortcut else 1, None, N, cin, cout, g1, d, h, w, st)
        pw1 = A.alloc(P * cout * (cin // g1) * 27)
        self._call("l3u_gconv3_bwd_weight", dy1.data_ptr(), cout * S, x.p, x.ns, None, A.ptr(pw1),
                   N, cin, cout, g1, d, h, w, st)
        n1w = cout * (cin // g1) * 27
        self._seg(pw1, P, n1w, 1, n1w, n1)
        if shortcut:
            self._pw_bwd(flat, drv, None, x, pre + "shortcut.0.weight", dxv, 1, N, S, st)
        if self.debug is not None and not self._dry:
            self.debug[pre + "#"] = {"dy2": dy2, "dr": drv, "dy1": dy1, "dx": dxv}

    def _block_bwd(self, flat, pre, sv, dout, dxv, st, dev):
        """Backward of ResidualBlock.forward (unet3d.py:77-93).  Writes d(block input) into dxv
        (overwrite) and records the block's weight-gradient reductions."""
        if self.kinds[pre][0][0] != "ds":
            return self._block_bwd_g(flat, pre, sv, dout, dxv, st, dev)
        A = self.bwd_arena
        x, out, recs = sv["x"], sv["out"], sv["recs"]
        if self.debug is not None and not self._dry:
            self.debug[pre] = dout
        d, h, w = sv["dims"]
        S = d * h * w
        N = x.t.shape[0]
        cin, cout = x.C, out.C
        e = lambda *s: self._empty(*s, device=dev)  # noqa: E731
        rec_r, rec1, rec2 = recs[0].data_ptr(), recs[1].data_ptr(), recs[2].data_ptr()
        shortcut = sv["shortcut"]
        rv = sv["r"] if shortcut else x
        y2, z2, z1 = sv["y2"], sv["z2"], sv["z1"]
        y1v = sv.get("y1v") or V(sv["y1"], 0, cout * S, cout)   # rank-1: z1, negative stride
        # (1) block tail: out = lrelu(IN2(y2) + residual)
        fused = self._tail_fusable(sv, cin, cout, S)
        sc_done = False   # the shortcut's d(input) already written (paired with conv2's backward)
        dz2 = e(N, cout, S)
        if fused:
            # (1+2) the tail reduce, then conv2.pointwise backward with the tail's apply in its
            # prologue (dy2 is never written)
            pn, ntp = self._tail_bwd(pre, sv, dout, dxv, N, cout, S, st, dev, fused=True)
            if (_PAIR_BWD and shortcut and S <= _PAIR_TAIL_MAX_S
                    and (max(cin, cout) <= 2 * min(cin, cout)
                         or (_PAIR_TAIL_NARROW and max(cin, cout) <= 16))
                    and (sv["r"].scale is None or (_PAIR_TAIL_NARROW and max(cin, cout) <= 16))):
                # ... with the shortcut backward in the same launch (it writes d(input) first);
                # the column-block counts of the two may differ by 2x at most, a rank-1 shortcut
                # operand (the first block's) only beside a single column block
                self._pw_bwd_tail_pair(flat, dout, sv["out"], pn, ntp,
                                       (V(y2, 0, cout * S, cout), rec2, V(z2, 0, cout * S, cout),
                                        pre + "conv2.pointwise.weight", V(dz2, 0, cout * S, cout), 1),
                                       (sv["r"], rec_r, x, pre + "shortcut.0.weight", dxv, 2), N, S, st)
                sc_done = True
            else:
                self._pw_bwd_tail(flat, dout, sv["out"], V(y2, 0, cout * S, cout), rec2, pn, ntp, 1,
                                  V(z2, 0, cout * S, cout), pre + "conv2.pointwise.weight",
                                  V(dz2, 0, cout * S, cout), 0, N, S, st)
        else:
            dy2, drv = self._tail_bwd(pre, sv, dout, dxv, N, cout, S, st, dev)
            # (2) conv2.pointwise backward; at the 12^3 / 6^3 levels paired in one launch with the
            # shortcut backward (both read the tail's outputs), which then writes d(input) first
            if (_PAIR_BWD and shortcut and nat.query("l3u_pw_bwd2_supported", cout, S)
                    and nat.query("l3u_pw_bwd_supported", cout, cin, S)):
                self._pw_bwd2(flat, (V(dy2, 0, cout * S, cout), V(z2, 0, cout * S, cout),
                                     pre + "conv2.pointwise.weight", V(dz2, 0, cout * S, cout)),
                              (drv, x, pre + "shortcut.0.weight", dxv), N, S, st)
                sc_done = True
            else:
                self._pw_bwd(flat, V(dy2, 0, cout * S, cout), None, V(z2, 0, cout * S, cout),
                             pre + "conv2.pointwise.weight", V(dz2, 0, cout * S, cout), 0, N, S, st)
        # (3) conv2.depthwise backward fused with LeakyReLU/Dropout/IN1 backward partials
        nch = nat.query("l3u_dw3_nchunk", N, cout, d, h, w)
        pd2 = A.alloc(cout * N * nch * 27)
        pi1 = A.alloc(2 * cout * N * nch * 2)          # fp64 partials
        pid = pi1 // 2
        dpre = e(N, cout, S)
        self._call("l3u_dw3_bwd", dz2.data_ptr(), cout * S, y1v.p, y1v.sns,
                   self._w(flat, pre + "conv2.depthwise.weight"), rec1, dpre.data_ptr(), cout * S, 0,
                   A.ptr(pd2), A.ptr(pi1), N, cout, d, h, w, st)
        self._seg_dw(pd2, N * nch, cout, pre + "conv2.depthwise.weight")
        self._seg(pid + 1, N * nch, 2, N * nch * 2, cout, pre + "norm1.weight", f64=1)
        self._seg(pid + 0, N * nch, 2, N * nch * 2, cout, pre + "norm1.bias", f64=1)
        # (4) conv1.pointwise backward, with the IN1 backward (dy1 from dpre) folded in when the
        # fused kernel takes the shape
        dz1 = e(N, cin, S)
        dpv = V(dpre, 0, cout * S, cout)
        name1 = pre + "conv1.pointwise.weight"
        if nat.query("l3u_pw_bwd_supported", cout, cin, S):
            self._pw_bwd(flat, dpv, (y1v.p, y1v.sns, rec1, A.ptr(pi1), nch),
                         V(z1, 0, cin * S, cin), name1, V(dz1, 0, cin * S, cin), 0, N, S, st)
        else:
            assert y1v.scale is None
            self._call("l3u_in_bwd_apply", dpre.data_ptr(), cout * S, y1v.p, y1v.ns, rec1,
                       A.ptr(pi1), nch, dpre.data_ptr(), cout * S, N, cout, S, st)
            self._pw_bwd(flat, dpv, None, V(z1, 0, cin * S, cin), name1, V(dz1, 0, cin * S, cin), 0,
                         N, S, st)
        dy1 = dpre
        # (5) conv1.depthwise backward: writes d(input) (Conv1x1 shortcut) or accumulates into the
        # identity-shortcut gradient (or the paired shortcut's) already there; a + b == b + a, so
        # the order of the two terms does not change a bit
        nch1 = nat.query("l3u_dw3_nchunk", N, cin, d, h, w)
        pd1 = A.alloc(cin * N * nch1 * 27)
        self._call("l3u_dw3_bwd", dz1.data_ptr(), cin * S, x.p, x.ns,
                   self._w(flat, pre + "conv1.depthwise.weight"), None, dxv.p, dxv.ns,
                   0 if shortcut and not sc_done else 1, A.ptr(pd1), None, N, cin, d, h, w, st)
        self._seg_dw(pd1, N * nch1, cin, pre + "conv1.depthwise.weight")
        # (6) shortcut conv backward accumulates into d(input)
        if sc_done:
            pass
        elif fused:
            self._pw_bwd_tail(flat, dout, sv["out"], sv["r"], rec_r, pn, ntp, 2, x,
                              pre + "shortcut.0.weight", dxv, 1, N, S, st)
        elif shortcut:
            self._pw_bwd(flat, drv, None, x, pre + "shortcut.0.weight", dxv, 1, N, S, st)
        if self.debug is not None and not self._dry:
            self.debug[pre + "#"] = {"dz2": dz2, "dy1": dy1, "dz1": dz1, "dx": dxv}
            if not fused:
                self.debug[pre + "#"].update(dy2=dy2, dr=drv)

    def _pw_bwd(self, flat, dy, pro, x, name, dx, accumulate, N, S, st):
        """Backward of a 1x1 conv y = W x (W = parameter `name`, [J][K]): dx (+)= W^T dy, and the
        weight-gradient partials recorded for the reduction into gflat[name].
        pro = (y, y_nstride, rec, in_part, npart): dy holds dpre of the preceding InstanceNorm
        and the fused kernel applies its backward on the fly."""
        J, K = dy.C, x.C
        w = self._w(flat, name)
        A = self.bwd_arena
        if nat.query("l3u_pw_bwd_supported", J, K, S):
            npw = nat.query("l3u_pw_bwd_nparts", N, J, K, S)
            part = A.alloc(npw * J * K)
            y, yns, rec, ip, npart = pro if pro is not None else (None, 0, None, None, 0)
            self._call("l3u_pw_bwd", dy.p, dy.ns, y, yns, rec, ip, npart, x.p, x.ns, w, dx.p, dx.ns,
                       accumulate, A.ptr(part), N, J, K, S, st)
        else:
            assert pro is None
            npw = nat.query("l3u_pw_bwd_weight_nparts", N, S)
            part = A.alloc(npw * J * K)
            self._call32("l3u_pw_fwd", dy.p, dy.ns, w, 1, None, dx.p, dx.ns, accumulate, None, N, J,
                         K, S, st)
            self._call("l3u_pw_bwd_weight", dy.p, dy.ns, x.p, x.ns, A.ptr(part), N, J, K, S, st)
        self._seg(part, npw, J * K, 1, J * K, name)

    def _pw_bwd2(self, flat, a, b, N, S, st):
        """Two plain _pw_bwd calls (dy, x, weight name, dx) of the same J in one launch
        (l3u_pw_bwd2); both dx are overwritten."""
        A = self.bwd_arena
        J = a[0].C
        parts = []
        for dy, x, name, dx in (a, b):
            npw = nat.query("l3u_pw_bwd_nparts", N, J, x.C, S)
            parts.append((A.alloc(npw * J * x.C), npw, x.C, name))
        (dya, xa, _, dxa), (dyb, xb, _, dxb) = a, b
        self._call("l3u_pw_bwd2", dya.p, dya.ns, xa.p, xa.ns, self._w(flat, a[2]), dxa.p, dxa.ns, 0,
                   A.ptr(parts[0][0]), xa.C, dyb.p, dyb.ns, xb.p, xb.ns, self._w(flat, b[2]), dxb.p,
                   dxb.ns, 0, A.ptr(parts[1][0]), xb.C, N, J, S, st)
        for off, npw, K, name in parts:
            self._seg(off, npw, J * K, 1, J * K, name)

    def _pw_bwd_tail_pair(self, flat, dout, out, pn, ntp, a, b, N, S, st):
        """The two _pw_bwd_tail calls of a block (a, b = (yr, rec, x, weight name, dx, sel)) in one
        launch (l3u_pw_bwd_tail_pair); both dx are overwritten."""
        J = out.C
        A = self.bwd_arena
        args, segs = [], []
        for yr, rec, x, name, dx, sel in (a, b):
            npw = nat.query("l3u_pw_bwd_nparts", N, J, x.C, S)
            off = A.alloc(npw * J * x.C)
            segs.append((off, npw, J * x.C, name))
            args += [yr.p, yr.sns, rec, x.p, x.ns, self._w(flat, name), dx.p, dx.ns, 0, A.ptr(off), x.C,
                     sel]
        dscale = dout.scale
        if dout.pool is not None:
            dpool, idx, (d, h, w) = dout.pool
            pool = [dpool.data_ptr(), J * (S // 8), idx.data_ptr(), h, w]
        else:
            pool = [None, 0, None, 0, 0]
        self._call("l3u_pw_bwd_tail_pair", dout.p, dout.ns, dscale, *pool, out.p, out.ns, A.ptr(pn),
                   ntp, *args, N, J, S, st)
        for off, npw, n, name in segs:
            self._seg(off, npw, n, 1, n, name)

    def _pw_bwd_tail(self, flat, dout, out, yr, rec, pn, ntp, sel, x, name, dx, accumulate, N, S,
                     st):
        """_pw_bwd of conv2.pointwise (sel 1, yr = y2) or the shortcut (sel 2, yr = r) with the
        block tail's InstanceNorm/LeakyReLU backward formed in the kernel prologue."""
        J, K = out.C, x.C
        A = self.bwd_arena
        npw = nat.query("l3u_pw_bwd_nparts", N, J, K, S)
        part = A.alloc(npw * J * K)
        if dout.scale is not None:   # rank-1 dout (l3u_outconv_bwd_dz)
            self._call("l3u_pw_bwd_tail_r1", dout.p, dout.ns, dout.scale, out.p, out.ns, yr.p, yr.sns,
                       rec, A.ptr(pn), ntp, sel, x.p, x.ns, self._w(flat, name), dx.p, dx.ns,
                       accumulate, A.ptr(part), N, J, K, S, st)
        elif dout.pool is not None:   # skip gradient + the folded MaxPool3d backward
            dpool, idx, (d, h, w) = dout.pool
            self._call("l3u_pw_bwd_tail_up", dout.p, dout.ns, dpool.data_ptr(), J * (S // 8),
                       idx.data_ptr(), out.p, out.ns, yr.p, yr.sns, rec, A.ptr(pn), ntp, sel, x.p,
                       x.ns, self._w(flat, name), dx.p, dx.ns, accumulate, A.ptr(part), N, J, K, d, h,
                       w, st)
        else:
            self._call("l3u_pw_bwd_tail", dout.p, dout.ns, out.p, out.ns, yr.p, yr.sns, rec,
                       A.ptr(pn), ntp, sel, x.p, x.ns, self._w(flat, name), dx.p, dx.ns, accumulate,
                       A.ptr(part), N, J, K, S, st)
        self._seg(part, npw, J * K, 1, J * K, name)

    def _seg_dw(self, off, count, C, name):
        # dw_part layout [C][count][27] -> grad [C][27]
        for c in range(C):
            self._seg(off + c * count * 27, count, 27, 1, 27, name, dst_elem=c * 27)
