"""Reference of one online-training step (BASELINE config 5) for the GPU parity tests -- TEST
INFRASTRUCTURE, never imported by the product.

A plain restatement in float64 PyTorch (autograd) of:
  * tcnn pcg32 (random.h) and the training-pixel draw of generate_training_samples_nerf
    (testbed_nerf.cu:862-881; nerf_random_image_pos_training nerf_device.cuh:553-576; image_idx
    nerf_device.cuh:578-597) -- to recover each ray's target pixel and random background;
  * the target colour of compute_loss_kernel_train_nerf (testbed_nerf.cu:1090-1160: random bg,
    sRGB training space, premultiplied 8-bit texels via read_rgba common_device.cuh:803-835);
  * volume compositing + Huber loss (loss_and_gradient, nerf_device.cuh:100-117, 601-616) and its
    gradient w.r.t. the network outputs (testbed_nerf.cu:1209-1275), here by autograd instead of
    the reference's closed form -- the closed form IS that derivative, so this checks it;
  * NerfNetwork forward/backward (nerf_network.h:81-268): hash-grid encoding (the numpy
    restatement in test_oracle_numpy.py gives corner indices/weights), density MLP, SH, rgb MLP,
    no biases, ReLU -- param gradients by autograd given the device's dL/d(output).

The device computes in fp16 (activations, output gradients) with f32 accumulation; the tests
therefore compare with stated relative tolerances, not bit for bit.
"""
import numpy as np
import torch

from test_oracle_numpy import PRIMES, _np_level_params, _np_sh

MULT = 0x5851F42D4C957F2D
M64 = (1 << 64) - 1
N_MAX_RANDOM_SAMPLES_PER_RAY = 16   # nerf_device.cuh:40


class Pcg32:
    """tcnn pcg32 (PCG XSH-RR 64/32), restated from the published algorithm."""

    def __init__(self, initstate, initseq=1):
        self.state, self.inc = 0, ((initseq << 1) | 1) & M64
        self.next_uint()
        self.state = (self.state + initstate) & M64
        self.next_uint()

    def copy(self):
        r = Pcg32.__new__(Pcg32)
        r.state, r.inc = self.state, self.inc
        return r

    def next_uint(self):
        old = self.state
        self.state = (old * MULT + self.inc) & M64
        xs = (((old >> 18) ^ old) >> 27) & 0xFFFFFFFF
        rot = old >> 59
        return ((xs >> rot) | (xs << ((-rot) & 31))) & 0xFFFFFFFF

    def next_float(self):
        u = (self.next_uint() >> 9) | 0x3F800000
        return float(np.array([u], np.uint32).view(np.float32)[0] - np.float32(1.0))

    def advance(self, delta=1 << 32):
        cur_mult, cur_plus, acc_mult, acc_plus = MULT, self.inc, 1, 0
        while delta > 0:
            if delta & 1:
                acc_mult = (acc_mult * cur_mult) & M64
                acc_plus = (acc_plus * cur_mult + cur_plus) & M64
            cur_plus = ((cur_mult + 1) * cur_plus) & M64
            cur_mult = (cur_mult * cur_mult) & M64
            delta //= 2
        self.state = (acc_mult * self.state + acc_plus) & M64


def step_rng(seed, step):
    """Testbed::m_rng at training step `step`: pcg32(seed), one draw for the density-grid rng, then
    one default advance per step (testbed.cu:3654-3667, testbed_nerf.cu:3350)."""
    r = Pcg32(seed)
    r.next_uint()
    for _ in range(step):
        r.advance()
    return r


def _f32(x):
    return np.float32(x)


def srgb_to_linear(c):
    c = np.asarray(c, np.float64)
    return np.where(c <= 0.04045, c / 12.92, ((c + 0.055) / 1.055) ** 2.4)


def linear_to_srgb(c):
    c = np.asarray(c, np.float64)
    return np.where(c < 0.0031308, 12.92 * c, 1.055 * c ** 0.41666 - 0.055)


def ray_targets(ray_idx, n_rays, rng, images, random_bg=True):
    """(target sRGB rgb, background sRGB) per ray index (compute_loss_kernel_train_nerf 1090-1160)."""
    n_img, h, w = images.shape[:3]
    tgt = np.zeros((len(ray_idx), 3))
    bgs = np.zeros((len(ray_idx), 3))
    for k, i in enumerate(ray_idx):
        i = int(i)
        r = rng.copy()
        r.advance(i * N_MAX_RANDOM_SAMPLES_PER_RAY)
        img = ((i * n_img) // n_rays) % n_img
        u, v = _f32(r.next_float()), _f32(r.next_float())
        px = min(max(int(u * _f32(w)), 0), w - 1)
        py = min(max(int(v * _f32(h)), 0), h - 1)
        r.advance(1)   # motionblur_time
        bg = np.array([r.next_float(), r.next_float(), r.next_float()]) if random_bg else np.zeros(3)
        bg = linear_to_srgb(srgb_to_linear(bg))
        texel = images[img, py, px].astype(np.float64) / 255.0
        a = texel[3]
        if a > 0:
            rgb = linear_to_srgb(srgb_to_linear(texel[:3]))   # premultiply, unpremultiply, back to sRGB
            tgt[k] = rgb * a + (1 - a) * bg
        else:
            tgt[k] = bg
        bgs[k] = bg
    return tgt, bgs


def huber(d, alpha=0.1):
    """loss_and_gradient Huber (nerf_device.cuh:100-117), / 5 as in the reference's LossType::Huber."""
    ad = d.abs()
    return torch.where(ad > alpha, ad - 0.5 * alpha, 0.5 / alpha * d * d) / 5.0


def ray_loss_grad(out16, dt, target, bg, n_rays, loss_scale=128.0, eps=1e-4):
    """One ray: network outputs [n][4] (fp16 values) -> (compacted count, loss, dL/d(output) [cn][4]
    scaled by loss_scale / n_rays) -- without the density regularisers."""
    o = torch.tensor(np.asarray(out16, np.float64), requires_grad=True)
    dt = torch.tensor(np.asarray(dt, np.float64))
    rgb = torch.sigmoid(o[:, :3])
    alpha = 1.0 - torch.exp(-torch.exp(o[:, 3]) * dt)
    T = torch.ones((), dtype=torch.float64)
    acc = torch.zeros(3, dtype=torch.float64)
    cn = 0
    for j in range(o.shape[0]):
        if float(T.detach()) < eps:
            break
        acc = acc + alpha[j] * T * rgb[j]
        T = T * (1.0 - alpha[j])
        cn += 1
    if cn == o.shape[0]:
        acc = acc + T * torch.tensor(bg)
    loss = huber(acc - torch.tensor(target)).sum() / 3.0
    loss.backward()
    g = o.grad.detach().numpy()[:cn] * (loss_scale / n_rays) * 3.0   # the reference's gradient is of the per-channel sum
    return cn, float(loss) / n_rays, g


class TorchNetwork:
    """NerfNetwork forward in float64 torch with fp16 parameters (tcnn param order nerf_network.h:356-371)."""

    def __init__(self, cfg, params16):
        p = torch.tensor(np.asarray(params16, np.float16).astype(np.float64))
        self.cfg = cfg
        self.p = p.clone().requires_grad_(True)
        self.levels = _np_level_params(cfg)

    def corners(self, x):
        """per level: (indices [n][8] into the level, weights [n][8]) -- numpy restatement of the grid lookup"""
        F = self.cfg["n_features_per_level"]
        out = []
        for (off, size, scale, res) in self.levels:
            pf = (np.float64(scale) * x.astype(np.float64) + 0.5).astype(np.float32)
            fl = np.floor(pf)
            pg = fl.astype(np.int64)
            w = (pf - fl).astype(np.float32)
            idxs, ws = [], []
            for c in range(8):
                weight = np.ones(len(x), np.float32)
                pl = []
                for d in range(3):
                    if c & (1 << d):
                        weight = (weight * w[:, d]).astype(np.float32)
                        pl.append(pg[:, d] + 1)
                    else:
                        weight = (weight * (np.float32(1.0) - w[:, d])).astype(np.float32)
                        pl.append(pg[:, d])
                pl = [q.astype(np.uint64) for q in pl]
                if res ** 3 <= size:
                    index = (pl[0] + pl[1] * np.uint64(res) + pl[2] * np.uint64(res * res)) & np.uint64(0xFFFFFFFF)
                else:
                    index = ((pl[0] * PRIMES[0]) ^ (pl[1] * PRIMES[1]) ^ (pl[2] * PRIMES[2])) & np.uint64(0xFFFFFFFF)
                idxs.append(((index % np.uint64(size)).astype(np.int64) + off) * F)
                ws.append(weight.astype(np.float64))
            out.append((np.stack(idxs, 1), np.stack(ws, 1)))
        return out

    def forward(self, coords):
        """coords [n][7] -> (rgb raw [n][3], sigma raw [n]) as float64 tensors"""
        F = self.cfg["n_features_per_level"]
        grid = self.p[10240:]
        feats = []
        for idx, w in self.corners(coords[:, :3]):
            idx_t = torch.tensor(idx)
            w_t = torch.tensor(w)
            g = torch.stack([grid[idx_t + f] for f in range(F)], -1)   # [n][8][F]
            feats.append((w_t[..., None] * g).sum(1))
        enc = torch.cat(feats, 1)
        W = lambda a, n_out, n_in: self.p[a:a + n_out * n_in].reshape(n_out, n_in)
        h = torch.relu(enc @ W(0, 64, 32).T)
        dens = h @ W(2048, 16, 64).T
        sh = torch.tensor(_np_sh(coords[:, 4:7]).astype(np.float64))
        rin = torch.cat([dens, sh], 1)
        h = torch.relu(rin @ W(3072, 64, 32).T)
        h = torch.relu(h @ W(5120, 64, 64).T)
        out = h @ W(9216, 16, 64).T
        return out[:, :3], dens[:, 0]

    def param_grads(self, coords, dl_dout):
        """d(sum dL/dout * out)/d params for upstream gradients dl_dout [n][4] (rgb raw, sigma raw)"""
        if self.p.grad is not None:
            self.p.grad = None
        rgb, sig = self.forward(coords)
        g = torch.tensor(np.asarray(dl_dout, np.float64))
        (rgb * g[:, :3]).sum().add((sig * g[:, 3]).sum()).backward()
        return self.p.grad.detach().numpy()
