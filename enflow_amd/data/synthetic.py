"""Synthetic molecule batches shaped like the reference's datasets.

There is no network and no rdkit/OpenMM here, so the benchmark and tests use
compact random-walk "molecules" that go through the same preparation the
reference applies in BaseDataset._get_data + main.py's transforms
(enflow/data/base.py:211-239, enflow/main.py:74-80, enflow/data/transforms.py):

* positions in Angstrom; when no box is given the box is
  round(max - min) per axis of the FIRST molecule and is then reused for every
  molecule, exactly as BaseDataset caches ``self.box`` (base.py:212-213,
  helpers.get_box_len); converted to LJ units (ConvertPositionsFrom), then
  centred (Center).  Random walks whose extent is under ``min_extent`` along
  any axis are redrawn so that no box component can round to r_cut (a pair at
  exactly the cut-off distance makes the edge set depend on the last ulp);
* h = one-hot atom types over {H, C, N, O, F} (constants.atom_types),
  g ~ N(0, 1) (base.py:230), velocities ~ Maxwell-Boltzmann at `kelvin`
  (RandomizeVelocity: Gaussian components with variance kBT, m = 1);
* r_cut in Angstrom converted to LJ units.

Everything is float64 numpy, in the reference's concatenated-batch layout
plus ``mol_ptr`` CSR offsets (Data.N, base.py:34-50).
"""
import numpy as np

from ..utils.conversion import dist_to_lj, kelvin_to_lj, time_to_lj

# alanine-dipeptide-like composition (22 atoms: 12 H, 6 C, 2 N, 2 O)
_COMPOSITION = (12, 6, 2, 2, 0)


def _random_walk(n, rng, bond=1.5, min_sep=1.15, radius=4.0):
    pts = np.zeros((n, 3))
    for a in range(1, n):
        best = None
        for _ in range(200):
            d = rng.normal(size=3)
            d *= bond / np.linalg.norm(d)
            p = pts[a - 1] + d
            if np.linalg.norm(p) > radius:
                continue
            if np.min(np.linalg.norm(pts[:a] - p, axis=1)) < min_sep:
                continue
            best = p
            break
        if best is None:
            d = rng.normal(size=3)
            best = pts[a - 1] + d * bond / np.linalg.norm(d)
        pts[a] = best
    return pts


def _types(n, rng):
    comp = np.array(_COMPOSITION, dtype=np.float64)
    counts = np.floor(comp / comp.sum() * n).astype(int)
    counts[0] += n - counts.sum()
    t = np.repeat(np.arange(len(comp)), counts)
    rng.shuffle(t)
    return t


def make_molecules(num_mols, n_atoms=22, nf=5, seed=0, r_cut_ang=3.0,
                   box_ang=None, kelvin=300.0, radius=4.0, min_extent=4.6, chain=False):
    """Return a dict batch: h, g, pos, vel, box [A,3], r_cut [M], mol_ptr [M+1].

    ``n_atoms`` is an int or a per-molecule sequence (ragged batch).
    ``chain=True``: unconfined self-avoiding random walks (BASELINE configs[4]'s
    long chains) instead of compact ones.
    """
    if chain:
        radius = np.inf
    rng = np.random.default_rng(seed)
    sizes = [int(n_atoms)] * num_mols if np.isscalar(n_atoms) else [int(x) for x in n_atoms]
    assert len(sizes) == num_mols
    kBT = kelvin_to_lj(kelvin)
    hs, gs, ps, vs, bs = [], [], [], [], []
    box_a = None
    if box_ang is not None:
        box_a = np.broadcast_to(np.asarray(box_ang, dtype=np.float64), (3,)).copy()
    for n in sizes:
        for _ in range(100):
            pos_a = _random_walk(n, rng, radius=radius)
            if n < 8 or np.all(pos_a.max(0) - pos_a.min(0) >= min_extent):
                break
        if box_a is None:
            box_a = np.round(pos_a.max(0) - pos_a.min(0))          # get_box_len
            box_a = np.maximum(box_a, 5.0)
        pos = dist_to_lj(pos_a, 'ang')
        pos = pos - pos.mean(axis=0, keepdims=True)                 # Center
        t = _types(n, rng)
        h = np.zeros((n, nf))
        h[np.arange(n), np.minimum(t, nf - 1)] = 1.0
        hs.append(h)
        gs.append(rng.normal(size=(n, nf)))
        ps.append(pos)
        vs.append(rng.normal(scale=np.sqrt(kBT), size=(n, 3)))
        bs.append(np.repeat(dist_to_lj(box_a, 'ang')[None, :], n, axis=0))
    mol_ptr = np.zeros(num_mols + 1, dtype=np.int64)
    mol_ptr[1:] = np.cumsum(sizes)
    return dict(h=np.concatenate(hs), g=np.concatenate(gs), pos=np.concatenate(ps),
                vel=np.concatenate(vs), box=np.concatenate(bs),
                r_cut=np.full(num_mols, dist_to_lj(r_cut_ang, 'ang')),
                mol_ptr=mol_ptr)


def arrange_points_on_grid(n, box, gap):
    """n points on a regular grid inside [gap, box - gap] (the LJ dataset's
    start configuration, enflow/data/lj.py:9-28)."""
    num_z = int(np.ceil(n ** (1 / 3)))
    num_y = int(np.ceil((n / num_z) ** 0.5))
    num_x = int(np.ceil(n / (num_y * num_z)))
    x = np.linspace(gap, box[0] - gap, num_x)
    y = np.linspace(gap, box[1] - gap, num_y)
    z = np.linspace(gap, box[2] - gap, num_z)
    xv, yv, zv = np.meshgrid(x, y, z)
    return np.stack((xv.flatten(), yv.flatten(), zv.flatten()), axis=-1)[:n]


def make_lj_systems(n_atoms, num_systems=1, density=0.8, r_cut=2.5, nf=5, seed=0, kelvin=120.0,
                    jitter=0.15):
    """Periodic Lennard-Jones boxes shaped like the reference's LJ dataset
    (enflow/data/lj.py + simulated.py:36-76; example/generate.yaml: one
    2944-atom box), in LJ units: atoms on the start grid plus a random
    displacement (a thermalised liquid instead of an OpenMM trajectory,
    which needs openmm), wrapped into the box (apply_pbc) and centred;
    h, g ~ N(0, 1/sqrt(kBT)) (simulated.py:56-58), Maxwell-Boltzmann
    velocities.  ``n_atoms``: int or per-system sequence; box edge
    (n / density)^(1/3)."""
    rng = np.random.default_rng(seed)
    sizes = [int(n_atoms)] * num_systems if np.isscalar(n_atoms) else [int(x) for x in n_atoms]
    kBT = kelvin_to_lj(kelvin)
    hs, gs, ps, vs, bs = [], [], [], [], []
    for n in sizes:
        L = (n / density) ** (1.0 / 3.0)
        box = np.array([L, L, L])
        pos = arrange_points_on_grid(n, box, 0.5) + rng.uniform(-jitter, jitter, size=(n, 3))
        pos = pos - np.round(pos / box) * box                     # apply_pbc
        pos = pos - pos.mean(axis=0, keepdims=True)               # Center
        hs.append(rng.normal(0, 1 / np.sqrt(kBT), size=(n, nf)))
        gs.append(rng.normal(0, 1 / np.sqrt(kBT), size=(n, nf)))
        ps.append(pos)
        vs.append(rng.normal(scale=np.sqrt(kBT), size=(n, 3)))
        bs.append(np.repeat(box[None, :], n, axis=0))
    mol_ptr = np.zeros(len(sizes) + 1, dtype=np.int64)
    mol_ptr[1:] = np.cumsum(sizes)
    return dict(h=np.concatenate(hs), g=np.concatenate(gs), pos=np.concatenate(ps), vel=np.concatenate(vs),
                box=np.concatenate(bs), r_cut=np.full(len(sizes), float(r_cut)), mol_ptr=mol_ptr)


def default_dt(ps=1.0):
    """dynamics.dt = 1 ps converted like main.py:113."""
    return time_to_lj(ps, 'pico')


def default_kBT(kelvin=300.0):
    return kelvin_to_lj(kelvin)
