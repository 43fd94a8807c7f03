"""Lockstep model of the camera-ray workgroup schedules (analysis only):
per-pixel walk steps of the C3 frame (ort_debug_walk_steps over every 8x8 block, saved by
tools/order_model_steps.py as /tmp/sim/steps_<tag>.npy for the default camera and turned ones)
replayed under the tile-pair kernel's schedules: cost order from hints (a stable sort of the
pair's 512 slots by hint >> 1 into 8 blocks; wave w walks blocks 7-w and w; a wave costs the
longest walk of each block plus a shade/new-ray batch per block), no order (each wave its two
8x8 blocks), and an in-workgroup refill kernel (lanes refill from the pair's queue once R of
a wave's 64 are idle, each refill a batch).  Units: lockstep walk iterations.
Output: profiles/r05_order_model_c3.log."""
import numpy as np, sys
st = np.load('/tmp/sim/steps_static.npy'); mv = np.load('/tmp/sim/steps_yaw05.npy'); mv2 = np.load('/tmp/sim/steps_yaw2.npy')
H, W = st.shape
REF = 1.6  # cost of a shade + new camera ray + walk setup batch, in walk-step iterations
def pairs(img):
    # yields (512,) arrays in natural slot order: tile j, wave-block w, lane
    Hp, Wp = (H // 16) * 16, (W // 32) * 32
    a = img[:Hp, :Wp].reshape(Hp // 16, 2, 8, Wp // 32, 2, 2, 8)  # by, rowblk(wave>>1), ly, pairx, tile j, colblk(wave&1), lx
    # order: pair (by, pairx), j, wave=(rowblk*2+colblk), lane=(ly*8+lx)
    a = a.transpose(0, 3, 4, 1, 5, 2, 6).reshape(-1, 512)
    return a
def static_cost(c, h, ordered=True):
    n = c.shape[0]
    if ordered:
        b = np.minimum(h >> 1, 63)
        idx = np.argsort(b, axis=1, kind='stable')
        cs = np.take_along_axis(c, idx, 1).reshape(n, 8, 64)
    else:
        cs = c.reshape(n, 2, 4, 64).transpose(0, 2, 1, 3).reshape(n, 8, 64)  # wave w: tile0 block w, tile1 block w
        cs = cs.reshape(n, 4, 2, 64)
        m = cs.max(-1)
        return (m.sum(-1) + 2 * REF).sum()
    m = cs.max(-1)  # (n, 8)
    waves = m[:, ::-1][:, :4] + m[:, :4] + 2 * REF  # wave w: block 7-w and block w
    return waves.sum()
def refill_cost(c, R=16, order=None):
    tot = 0.0
    for q in range(c.shape[0]):
        cc = c[q] if order is None else c[q][order[q]]
        ptr = 256
        rem = [list(cc[w*64:(w+1)*64]) for w in range(4)]
        t = [REF] * 4
        active = [True]*4
        lanes = [np.array(cc[w*64:(w+1)*64], dtype=np.int64) for w in range(4)]
        # simulate each wave's iterations; the queue is shared: process waves in time order (approximate: round robin per iteration)
        while any(active):
            for w in range(4):
                if not active[w]: continue
                L = lanes[w]
                idle = int((L <= 0).sum())
                if idle == 64 and ptr >= 512:
                    active[w] = False; continue
                if idle >= R and ptr < 512:
                    take = min(idle, 512 - ptr)
                    ii = np.nonzero(L <= 0)[0][:take]
                    L[ii] = cc[ptr:ptr+take]; ptr += take
                    t[w] += REF
                    continue
                L -= 1
                t[w] += 1
        tot += sum(t)
    return tot
pc_st, pc_mv, pc_mv2 = pairs(st), pairs(mv), pairs(mv2)
useful = pc_st.sum() / 64
print('pairs', pc_st.shape[0])
a = static_cost(pc_st, pc_st); print('static perfect hints: %.4g  eff %.3f' % (a, useful / a))
b = static_cost(pc_mv, pc_st); print('moving 0.5deg stale:  %.4g  ratio %.3f' % (b, b / static_cost(pc_mv, pc_mv)))
b2 = static_cost(pc_mv2, pc_st); print('moving 2deg stale:    %.4g  ratio %.3f' % (b2, b2 / static_cost(pc_mv2, pc_mv2)))
c = static_cost(pc_st, None, ordered=False); print('no order:             %.4g  ratio %.3f' % (c, c / a))
sub = pc_st[::40]
for R in (8, 16, 32):
    r = refill_cost(sub, R); print('refill R=%d (sample 1/40): ratio to perfect %.3f' % (R, r / static_cost(sub, sub)))
print('--- shifted stale hints for the 0.5 deg turn (h(x) = static(x + s))')
for s_ in (-40, -26, -13, 0, 13, 26, 40):
    sh = np.roll(st, -s_, axis=1)
    print('shift %+d: ratio %.3f' % (s_, static_cost(pc_mv, pairs(sh)) / static_cost(pc_mv, pc_mv)))
# correlation of moved steps with shifted static
for s_ in (-26, 0, 26):
    sh = np.roll(st, -s_, axis=1)
    print('corr shift %+d: %.3f' % (s_, np.corrcoef(mv[:, 100:-100].ravel(), sh[:, 100:-100].ravel())[0, 1]))
print('--- hints aggregated over the previous frames of a 0.5 deg/frame turn (frame 2.5 deg)')
fr = [np.load(f'/tmp/sim/steps_{t}.npy') for t in ('static', 'yaw05', 'yaw1', 'yaw15', 'yaw2', 'yaw25')]
P = [pairs(f) for f in fr]
cur, best = P[5], static_cost(P[5], P[5])
print('stale (prev frame): %.3f' % (static_cost(cur, P[4]) / best))
for a in (0.3, 0.5, 0.7):
    h = fr[0].astype(np.float64)
    for k in range(1, 5):
        h = a * fr[k] + (1 - a) * h
    print('EMA alpha %.1f: %.3f' % (a, static_cost(cur, pairs(np.rint(h).astype(np.int64))) / best))
print('mean of 5: %.3f' % (static_cost(cur, pairs(np.rint(np.mean(fr[:5], axis=0)).astype(np.int64))) / best))
