"""Developer tool: one pixel of the 1200x675 final scene traced in the Python oracle
(oracle/pyoracle.py, the reference restated), every segment classified (sphere, material,
total internal reflection), TIR runs grouped by how they end. usage: python
tools/trace_pixel.py X Y [S]  (round 5: pixel (567, 308), the N=8 rank-4 chain)"""
import sys, math, collections
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
import oracle.pyoracle as po
SEED = 1764892800000
cam, objs = po.scene_builtin("complex", SEED, 675, 1200, 50)
X, Y = int(sys.argv[1]), int(sys.argv[2])
S = int(sys.argv[3]) if len(sys.argv) > 3 else 23
offsets = po.offset_lattice(cam.pixel_delta_v, cam.pixel_delta_u, S)
parent = po.XorShift(SEED)
for p in range(Y * cam.width + X):
    parent.copy_reset()
rnd = parent.copy_reset()
def hit_idx(o, d):
    best = None
    for i, obj in enumerate(objs):
        h = po.sphere_hit(obj[0], obj[1], o, d)
        if h is not None and (best is None or h[0] < best[0][0]):
            best = (h, i)
    return best
events = []  # per sample: list of (sphere idx or -1, kind, tir)
for off in offsets:
    o, d = po.get_ray(cam, X, Y, off, rnd)
    ev = []
    for depth in range(cam.max_depth):
        hb = hit_idx(o, d)
        if hb is None:
            ev.append((-1, 'sky', False)); break
        rec, i = hb
        m = objs[i][2]
        tir = False
        if m[0] == po.DIELECTRIC:
            _, p, normal, front = rec
            ratio = 1.0 / m[3] if front else m[3]
            ud = po.unit(d)
            cos_t = po.fmin(po.dot(po.neg(ud), normal), 1.0)
            tir = ratio * math.sqrt(1.0 - cos_t * cos_t) > 1.0
        ev.append((i, m[0], tir))
        o, d, att = po.scatter(m, d, rec, rnd)
    else:
        ev.append((None, 'cap', False))
    events.append(ev)
segs = sum(len([e for e in ev if e[0] is not None and e[1] != 'sky']) + (1 if ev[-1][1] == 'sky' else 0) for ev in events)
print("pixel", X, Y, "samples", len(events), "segments~", segs)
# TIR runs: consecutive TIR bounces in the same sphere; what ends them
runs = collections.Counter(); ends = collections.Counter(); tir_segs = 0; lens = []
hits = collections.Counter()
for ev in events:
    for e in ev:
        if e[0] is not None and e[0] >= 0: hits[e[0]] += 1
    k = 0
    while k < len(ev):
        e = ev[k]
        if e[2]:
            j = k
            while j < len(ev) and ev[j][2] and ev[j][0] == e[0]:
                j += 1
            L = j - k; tir_segs += L; lens.append(L)
            nxt = ev[j] if j < len(ev) else None
            ends[('sphere', e[0], 'then', None if nxt is None else (nxt[0], nxt[1] if not isinstance(nxt[1], int) else ['L','M','D'][nxt[1]], nxt[2]))] += 1
            k = j
        else:
            k += 1
print("TIR bounces", tir_segs, "runs", len(lens), "mean run", sum(lens)/max(1,len(lens)), "max", max(lens) if lens else 0)
print("top hit spheres", hits.most_common(6))
for k, v in ends.most_common(12):
    print(v, k)
caps = sum(1 for ev in events if ev[-1][1] == 'cap')
print("samples ending at depth cap", caps)
