"""ctypes binding of the fused fp32 MFMA TD3 learner (include/hockey_learner.h, csrc/hk_learner.hip).

``FusedLearner(agent, ring, batch)`` performs ``agent``'s learner updates (rl/td3/learner.py:55-218: clipped
double-Q target with policy smoothing, weighted smooth-L1 critic loss, delayed actor update, Polyak averaging, Adam
with the config's lr / eps 1e-6 / weight decay) on ``ring`` with a handful of HIP kernels per update instead of a few
hundred PyTorch ops.  The agent's modules stay the parameter owners (checkpoints, evaluation and acting use them
unchanged); their parameters are re-pointed into one flat buffer per network so that Polyak averaging is one launch.

Randomness is drawn by torch in the eager update's order -- the sampled slots (``ring.sample_indices``) and then the
target noise ``torch.randn_like`` of shape [B, 4] -- so from the same generator state a fused update consumes exactly
the eager update's random numbers (tests/test_gpu_learner.py compares the two).  The optimiser state is the
learner's own (Adam moments in fp32 device buffers): ``agent.opt_critic`` / ``opt_actor`` are not used.

Every call is asynchronous on torch's current stream and graph-capturable (fixed buffers, device step counters).
There is no CPU path: construction fails loudly without the library or a GPU.
"""
import ctypes
import os

import torch

from . import _native

LIB_PATH = os.environ.get("HK_LEARNER_LIB") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "_lib",
                                                            "libhockey_learner.so")
PACK_FLOATS = 16 * 64 * 8 + 2 * 16 * 16 * 64 * 4 + 16 * 64 * 4 + 256 * 4
MAX_SEG = 12
CHUNK = 256  # batch granularity (include/hockey_learner.h)
XP = 32

vp = ctypes.c_void_p


class Net(ctypes.Structure):
    _fields_ = [("w1", vp), ("b1", vp), ("w2", vp), ("b2", vp), ("w3", vp), ("b3", vp), ("pack", vp),
                ("n_in", ctypes.c_int32), ("n_out", ctypes.c_int32)]


class CriticIO(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int64), ("idx", vp), ("ring_s", vp), ("ring_a", vp), ("ring_r", vp),
                ("ring_s2", vp), ("ring_d", vp), ("noise", vp), ("iw", vp), ("target_actor", Net),
                ("target_q", Net * 2), ("q", Net * 2), ("gamma", ctypes.c_float), ("act_low", ctypes.c_float * 4),
                ("act_range", ctypes.c_float * 4), ("x0", vp), ("h1", vp * 2), ("dz1", vp * 2), ("dz2", vp * 2),
                ("p_db1", vp * 2), ("p_db2", vp * 2), ("p_dw3", vp * 2), ("p_db3", vp * 2), ("p_loss", vp),
                ("td", vp), ("sample_counter", vp)]


class SampleIO(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int64), ("seed", ctypes.c_uint64), ("counter", vp), ("size", vp), ("idx", vp),
                ("noise", vp), ("scale", ctypes.c_float), ("clip", ctypes.c_float)]


class ActorIO(ctypes.Structure):
    _fields_ = [("batch", ctypes.c_int64), ("idx", vp), ("ring_s", vp), ("actor", Net), ("q1", Net),
                ("act_low", ctypes.c_float * 4), ("act_range", ctypes.c_float * 4), ("x0", vp), ("h1", vp),
                ("h2", vp), ("dz1", vp), ("dz2", vp), ("p_db1", vp), ("p_db2", vp), ("p_dw3", vp), ("p_db3", vp),
                ("p_loss", vp)]


class WgJob(ctypes.Structure):
    _fields_ = [("dz", vp), ("x", vp), ("slab", vp), ("bias_slab", vp)]


class Seg(ctypes.Structure):
    _fields_ = [("param", vp), ("m", vp), ("v", vp), ("src", vp), ("rows", ctypes.c_int32), ("cols", ctypes.c_int32),
                ("ld", ctypes.c_int64), ("chunks", ctypes.c_int32), ("stride", ctypes.c_int64), ("target", vp)]


class AdamIO(ctypes.Structure):
    _fields_ = [("seg", Seg * MAX_SEG), ("n_seg", ctypes.c_int32), ("lr", ctypes.c_float), ("beta1", ctypes.c_float),
                ("beta2", ctypes.c_float), ("eps", ctypes.c_float), ("wd", ctypes.c_float), ("step", vp),
                ("loss_src", vp), ("loss_chunks", ctypes.c_int32), ("loss_scale", ctypes.c_float),
                ("loss_sum", vp), ("loss_count", vp), ("polyak", ctypes.c_int32), ("polyak_rho", ctypes.c_float),
                ("polyak_tau", ctypes.c_float)]


EXPORTS = ["hkl_last_error", "hkl_pack_floats", "hkl_pack", "hkl_critic_step", "hkl_actor_step", "hkl_wgrad",
           "hkl_wgrad_pair",
           "hkl_adam", "hkl_polyak", "hkl_tanh_probe", "hkl_sample"]


def tanh_probe(x):
    """The fused kernels' tanh of a device float32 tensor (accuracy check)."""
    x = x.contiguous().float()
    y = torch.empty_like(x)
    _check(lib().hkl_tanh_probe(_p(x), _p(y), x.numel(),
                                ctypes.c_void_p(torch.cuda.current_stream(x.device).cuda_stream)), "hkl_tanh_probe")
    return y
_lib = None


def lib():
    """The loaded learner library; raises HockeyNativeError if it is missing (no CPU fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise _native.HockeyNativeError(
                f"{LIB_PATH} not found: build it with `make -C hockey-env_amd/csrc` (hipcc, gfx950)")
        L = ctypes.CDLL(LIB_PATH)
        L.hkl_last_error.restype = ctypes.c_char_p
        L.hkl_pack.argtypes = [ctypes.POINTER(Net), ctypes.c_int, vp, vp]
        L.hkl_critic_step.argtypes = [ctypes.POINTER(CriticIO), vp]
        L.hkl_actor_step.argtypes = [ctypes.POINTER(ActorIO), vp]
        L.hkl_wgrad.argtypes = [ctypes.POINTER(WgJob), ctypes.c_int, ctypes.c_int, ctypes.c_int64, vp]
        L.hkl_wgrad_pair.argtypes = [ctypes.POINTER(WgJob), ctypes.c_int, ctypes.POINTER(WgJob), ctypes.c_int,
                                     ctypes.c_int64, vp]
        L.hkl_adam.argtypes = [ctypes.POINTER(AdamIO), vp]
        L.hkl_polyak.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_float, ctypes.c_float, vp]
        L.hkl_tanh_probe.argtypes = [vp, vp, ctypes.c_int64, vp]
        L.hkl_sample.argtypes = [ctypes.POINTER(SampleIO), vp]
        if L.hkl_pack_floats() != PACK_FLOATS:
            raise _native.HockeyNativeError("libhockey_learner.so pack size differs from hockey_amd.learner_hip")
        _lib = L
    return _lib


def _check(rc, what):
    if rc != 0:
        raise _native.HockeyNativeError(f"{what} failed ({rc}): {lib().hkl_last_error().decode()}")


def _p(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def flatten_(module):
    """Re-point every parameter of ``module`` into one contiguous fp32 buffer (values unchanged); returns it."""
    params = list(module.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in params]).contiguous()
    o = 0
    for p in params:
        n = p.numel()
        p.data = flat[o:o + n].view_as(p)
        o += n
    return flat


def _mlp_layers(m):
    """(fc1, fc2, fc3) of an Actor / _QNet."""
    return m.fc1, m.fc2, m.fc3


class _NetBufs:
    """One MLP's parameter pointers and its MFMA operand pack."""

    def __init__(self, m, device):
        self.m = m
        self.pack = torch.zeros(PACK_FLOATS, dtype=torch.float32, device=device)
        f1, f2, f3 = _mlp_layers(m)
        self.net = Net(_p(f1.weight), _p(f1.bias), _p(f2.weight), _p(f2.bias), _p(f3.weight), _p(f3.bias),
                       _p(self.pack), f1.in_features, f3.out_features)


class FusedLearner:
    """Learner updates of ``agent`` (hockey_amd.td3.TD3) on ``ring`` at batch ``batch`` (a multiple of 256) with the
    fused kernels; same interface as the eager path: ``update(train_actor, acc)``."""

    def __init__(self, agent, ring, batch, rng="device", seed=None):
        L = lib()
        if rng not in ("device", "torch"):
            raise ValueError("rng must be 'device' or 'torch'")
        self.rng = rng
        self.L = L
        self.agent, self.ring, self.B = agent, ring, int(batch)
        if getattr(agent, "_fused_learner", None) is not None:
            raise RuntimeError("FusedLearner: this agent already has a fused learner (one owns its Adam state)")
        dev = agent.device
        if dev.type != "cuda":
            raise _native.HockeyNativeError("the fused learner runs on the GPU only")
        if self.B <= 0 or self.B % CHUNK:
            raise ValueError(f"fused learner batch must be a positive multiple of {CHUNK}, got {self.B}")
        if agent.actor.fc1.out_features != 256:
            raise ValueError("fused learner: hidden width 256 only (rl/td3/networks.py h)")
        B, G = self.B, self.B // 64
        C = self.B // (512 if self.B % 512 == 0 else 256)  # hkl_wgrad's split-K chunks: the critics' dW2 (2 jobs)
        CA = self.B // 256  # the actor's dW2 (one k-width-256 job: 256-sample chunks, include/hockey_learner.h)
        C1 = self.B // 256  # dW1 (k width 32)
        c = agent.cfg
        self.cfg = c
        self.flat = {k: flatten_(getattr(agent, k)) for k in ("actor", "critic", "target_actor", "target_critic")}
        self.m = {k: torch.zeros_like(self.flat[k]) for k in ("actor", "critic")}
        self.v = {k: torch.zeros_like(self.flat[k]) for k in ("actor", "critic")}
        self.step = {k: torch.zeros((), dtype=torch.int64, device=dev) for k in ("actor", "critic")}
        self.nets = {"actor": _NetBufs(agent.actor, dev), "target_actor": _NetBufs(agent.target_actor, dev),
                     "q1": _NetBufs(agent.critic.q1, dev), "q2": _NetBufs(agent.critic.q2, dev),
                     "tq1": _NetBufs(agent.target_critic.q1, dev), "tq2": _NetBufs(agent.target_critic.q2, dev)}
        z = lambda *shape: torch.zeros(shape, dtype=torch.float32, device=dev)  # noqa: E731
        self.buf = {"x0": z(B, XP), "x0a": z(B, XP), "td": z(B), "noise": z(B, 4), "loss_c": z(G), "loss_a": z(G)}
        for k in ("h1", "dz1", "dz2"):
            self.buf[k] = [z(B, 256), z(B, 256)]
            self.buf[k + "a"] = z(B, 256)
        self.buf["h2a"] = z(B, 256)
        for k in ("db1", "db2", "dw3"):
            self.buf["p_" + k] = [z(G, 256), z(G, 256)]
        self.buf["p_db3"] = [z(G), z(G)]
        self.buf["pa_db1"], self.buf["pa_db2"] = z(G, 256), z(G, 256)
        self.buf["pa_dw3"], self.buf["pa_db3"] = z(G, 4, 256), z(G, 4)
        self.buf["s_w2"] = [z(C, 256, 256), z(C, 256, 256)]
        self.buf["s_w1"] = [z(C1, 256, XP), z(C1, 256, XP)]
        self.buf["s_b2"], self.buf["s_b1"] = [z(C, 256), z(C, 256)], [z(C1, 256), z(C1, 256)]
        self.buf["sa_w2"], self.buf["sa_w1"] = z(CA, 256, 256), z(C1, 256, XP)
        self.buf["sa_b2"], self.buf["sa_b1"] = z(CA, 256), z(C1, 256)
        self.idx = torch.zeros(B, dtype=torch.int64, device=dev)
        self.sample_counter = torch.zeros((), dtype=torch.int64, device=dev)
        sio = SampleIO()
        sio.batch = B
        sio.seed = (int(agent.seed if seed is None else seed) * 0x9E3779B97F4A7C15 + 0x4C4541524E) % (1 << 64)
        sio.counter, sio.size, sio.idx, sio.noise = (_p(self.sample_counter), _p(ring.size_t), _p(self.idx),
                                                     _p(self.buf["noise"]))
        sio.scale, sio.clip = c.target_action_noise_scale, c.target_action_noise_clip
        self.sio = sio
        self.iw = z(B) if ring.prioritized else None
        low = agent.critic.action_low.float().cpu().tolist()
        rng = agent.critic.action_range.float().cpu().tolist()
        self._build_io(low, rng)
        # Adam adds each step's loss into a device accumulator: a private one until the caller sets its own, so
        # that an update never runs with the loss pointers unset
        self.set_loss_accumulator(torch.zeros(4, dtype=torch.float64, device=dev))
        st = self._stream()
        for group in (("actor", "target_actor"), ("q1", "q2"), ("tq1", "tq2")):
            self._pack([self.nets[k] for k in group], None, st)
        agent._fused_learner = self  # TD3.update / TD3.load now fail loudly (TD3._no_fused)

    # ------------------------------------------------------------------ structs (fixed pointers)
    def _build_io(self, low, rng):
        b, n = self.buf, self.nets
        cio = CriticIO()
        cio.batch, cio.idx = self.B, _p(self.idx)
        r = self.ring
        cio.ring_s, cio.ring_a, cio.ring_r, cio.ring_s2, cio.ring_d = _p(r.s), _p(r.a), _p(r.r), _p(r.s2), _p(r.d)
        cio.noise, cio.iw = _p(b["noise"]), _p(self.iw)
        cio.target_actor = n["target_actor"].net
        cio.target_q[0], cio.target_q[1] = n["tq1"].net, n["tq2"].net
        cio.q[0], cio.q[1] = n["q1"].net, n["q2"].net
        cio.gamma = self.cfg.gamma
        for i in range(4):
            cio.act_low[i], cio.act_range[i] = low[i], rng[i]
        cio.x0 = _p(b["x0"])
        for k in range(2):
            cio.h1[k], cio.dz1[k], cio.dz2[k] = _p(b["h1"][k]), _p(b["dz1"][k]), _p(b["dz2"][k])
            cio.p_db1[k], cio.p_db2[k] = _p(b["p_db1"][k]), _p(b["p_db2"][k])
            cio.p_dw3[k], cio.p_db3[k] = _p(b["p_dw3"][k]), _p(b["p_db3"][k])
        cio.p_loss, cio.td = _p(b["loss_c"]), _p(b["td"])
        cio.sample_counter = _p(self.sample_counter)
        self.cio = cio

        aio = ActorIO()
        aio.batch, aio.idx, aio.ring_s = self.B, _p(self.idx), _p(r.s)
        aio.actor, aio.q1 = n["actor"].net, n["q1"].net
        for i in range(4):
            aio.act_low[i], aio.act_range[i] = low[i], rng[i]
        aio.x0, aio.h1, aio.h2, aio.dz1, aio.dz2 = (_p(b["x0a"]), _p(b["h1a"]), _p(b["h2a"]), _p(b["dz1a"]),
                                                    _p(b["dz2a"]))
        aio.p_db1, aio.p_db2, aio.p_dw3, aio.p_db3 = _p(b["pa_db1"]), _p(b["pa_db2"]), _p(b["pa_dw3"]), _p(b["pa_db3"])
        aio.p_loss = _p(b["loss_a"])
        self.aio = aio
        G, C, C1 = self.B // 64, self.B // (512 if self.B % 512 == 0 else 256), self.B // 256
        CA = self.B // 256
        # Adam segments: torch parameter order of each network (fc1.w, fc1.b, fc2.w, fc2.b, fc3.w, fc3.b)
        self.adam = {}
        for name, nets, lr, wd, tau in (
                ("critic", [("q1", 0, "tq1"), ("q2", 1, "tq2")], self.cfg.lr_q, self.cfg.wd_q, self.cfg.tau_critic),
                ("actor", [("actor", None, "target_actor")], self.cfg.lr_pol, self.cfg.wd_pol, self.cfg.tau_actor)):
            io = AdamIO()
            segs = []
            flat, m, v = self.flat[name], self.m[name], self.v[name]
            tflat = self.flat["target_" + name]
            off = 0
            for key, k, tkey in nets:
                f1, f2, f3 = _mlp_layers(n[key].m)
                t1, t2, t3 = _mlp_layers(n[tkey].m)
                tparams = (t1.weight, t1.bias, t2.weight, t2.bias, t3.weight, t3.bias)
                if k is None:
                    srcs = [(b["sa_w1"], XP, C1, 256 * XP), (b["sa_b1"], 256, C1, 256), (b["sa_w2"], 256, CA, 65536),
                            (b["sa_b2"], 256, CA, 256), (b["pa_dw3"], 256, G, 1024), (b["pa_db3"], 4, G, 4)]
                else:
                    srcs = [(b["s_w1"][k], XP, C1, 256 * XP), (b["s_b1"][k], 256, C1, 256), (b["s_w2"][k], 256, C, 65536),
                            (b["s_b2"][k], 256, C, 256), (b["p_dw3"][k], 256, G, 256), (b["p_db3"][k], 1, G, 1)]
                for p, tp, (src, ld, chunks, stride) in zip((f1.weight, f1.bias, f2.weight, f2.bias, f3.weight,
                                                             f3.bias), tparams, srcs):
                    rows, cols = (p.shape[0], p.shape[1]) if p.dim() == 2 else (1, p.shape[0])
                    assert p.data_ptr() == flat.data_ptr() + off * 4, "parameters not in the flat buffer's order"
                    assert tp.data_ptr() == tflat.data_ptr() + off * 4 and tp.shape == p.shape, "target layout differs"
                    segs.append(Seg(_p(p), ctypes.c_void_p(m.data_ptr() + off * 4),
                                    ctypes.c_void_p(v.data_ptr() + off * 4), _p(src), rows, cols, ld, chunks, stride,
                                    _p(tp)))
                    off += p.numel()
            assert off == flat.numel()
            for i, s in enumerate(segs):
                io.seg[i] = s
            io.n_seg = len(segs)
            io.lr, io.beta1, io.beta2, io.eps, io.wd = lr, 0.9, 0.999, 1e-6, wd
            io.step = _p(self.step[name])
            io.loss_src = _p(b["loss_c"] if name == "critic" else b["loss_a"])
            io.loss_chunks = G
            io.loss_scale = (0.5 if name == "critic" else 1.0) / self.B
            # soft_update folded into the Adam launch (set per call: the critic's only on actor updates)
            io.polyak, io.polyak_rho, io.polyak_tau = 0, 1.0 - tau, tau
            self.adam[name] = io
        # weight-gradient jobs (one launch per k width): critics' dW2 / dW1 (+ b2 / b1), actor's
        J = lambda dz, x, sl, bs: WgJob(_p(dz), _p(x), _p(sl), _p(bs))  # noqa: E731
        self.wg = {"c256": (WgJob * 2)(*[J(b["dz2"][k], b["h1"][k], b["s_w2"][k], b["s_b2"][k]) for k in range(2)]),
                   "c32": (WgJob * 2)(*[J(b["dz1"][k], b["x0"], b["s_w1"][k], b["s_b1"][k]) for k in range(2)]),
                   "a256": (WgJob * 1)(J(b["dz2a"], b["h1a"], b["sa_w2"], b["sa_b2"])),
                   "a32": (WgJob * 1)(J(b["dz1a"], b["x0a"], b["sa_w1"], b["sa_b1"]))}

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.agent.device).cuda_stream)

    def _pack(self, bufs, step, st):
        arr = (Net * len(bufs))(*[x.net for x in bufs])
        _check(self.L.hkl_pack(arr, len(bufs), _p(step), st), "hkl_pack")

    def set_loss_accumulator(self, acc):
        """acc: float64 [4] = (sum critic loss, sum actor loss, critic updates, actor updates) on the device."""
        base = acc.data_ptr()
        self.adam["critic"].loss_sum, self.adam["critic"].loss_count = base, base + 16
        self.adam["actor"].loss_sum, self.adam["actor"].loss_count = base + 8, base + 24
        self._acc = acc

    # ------------------------------------------------------------------ one update
    def update(self, train_actor, idx=None, noise=None):
        """learner.update on a batch sampled from the ring: critic step, then (train_actor) the actor step and the
        Polyak averaging of both targets.  The batch's slots and target noise come from the device Philox stream
        (rng="device": one kernel), or from torch's generator in the eager learner's order (rng="torch": the slots
        via ring.sample_indices, then N(0, scale) [B, 4]), or (tests) from idx / noise: the slots and the UNCLIPPED
        N(0, scale) noise."""
        L, st, b = self.L, self._stream(), self.buf
        c = self.cfg
        prioritized = self.ring.prioritized
        if idx is None and noise is None and self.rng == "device" and not prioritized:
            _check(L.hkl_sample(ctypes.byref(self.sio), st), "hkl_sample")
            i = self.idx
        else:
            i = self.ring.sample_indices(self.B) if idx is None else idx
            self.idx.copy_(i)
            if noise is None:
                noise = torch.randn((self.B, 4), device=self.agent.device) * c.target_action_noise_scale
            b["noise"].copy_(torch.clamp(noise, -c.target_action_noise_clip, c.target_action_noise_clip))
        if self.iw is not None:
            wb = self.ring.w[i]
            p = wb / wb.sum()
            iw = (1.0 / (p * self.ring.size_t)) ** self.ring.beta
            self.iw.copy_(iw / iw.max())
        _check(L.hkl_critic_step(ctypes.byref(self.cio), st), "hkl_critic_step")
        _check(L.hkl_wgrad_pair(self.wg["c256"], 2, self.wg["c32"], 2, self.B, st), "hkl_wgrad_pair")
        # on an actor update the critic's soft_update runs here, with its Adam step: nothing later in the update
        # reads the target critic or changes the critic, so the values are those of soft_update at the end
        self.adam["critic"].polyak = 1 if train_actor else 0
        _check(L.hkl_adam(ctypes.byref(self.adam["critic"]), st), "hkl_adam")
        self._pack([self.nets["q1"], self.nets["q2"]], self.step["critic"], st)
        if self.ring.prioritized:
            self.ring.last = i
            self.ring.update_priorities(b["td"])
        if not train_actor:
            return
        _check(L.hkl_actor_step(ctypes.byref(self.aio), st), "hkl_actor_step")
        _check(L.hkl_wgrad_pair(self.wg["a256"], 1, self.wg["a32"], 1, self.B, st), "hkl_wgrad_pair")
        self.adam["actor"].polyak = 1  # the actor's soft_update with its Adam step
        _check(L.hkl_adam(ctypes.byref(self.adam["actor"]), st), "hkl_adam")
        self._pack([self.nets["actor"], self.nets["target_actor"], self.nets["tq1"], self.nets["tq2"]],
                   self.step["actor"], st)


def update_flops(batch, h=256, n_obs=18, n_act=4, policy_freq=2):
    """Algorithmic fp32 FLOPs of one learner update at ``batch`` (2 per multiply-add; averaged over the delayed actor
    update), counted from the layer shapes of rl/td3/networks.py: an MLP n_in -> h -> h -> n_out costs
    F(n_in, n_out) = n_in h + h h + h n_out MACs per sample forward; a backward to the first layer's input-side
    gradients costs h n_out + h h (data) and every weight gradient its forward MACs again.
      critic step: target actor + 2 target critics forward, 2 critics forward, 2 critics backward (data: W3^T, W2^T;
                   weights: dW1, dW2, dW3);
      actor step (every policy_freq-th): actor forward, Q1 forward, Q1 backward to its input (W3^T, W2^T, W1^T
                   action columns), actor backward (data and weights)."""
    fa, fc = n_obs * h + h * h + h * n_act, (n_obs + n_act) * h + h * h + h
    critic = fa + 2 * fc + 2 * fc + 2 * ((h + h * h) + fc)
    actor = fa + fc + ((h + h * h) + h * n_act) + ((h * n_act + h * h) + fa)
    return 2.0 * batch * (critic + actor / policy_freq)
