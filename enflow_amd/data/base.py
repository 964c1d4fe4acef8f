"""Batch container and neighbour-list handle (mirrors enflow/data/base.py:9-174).

``Data`` keeps the reference's fields and concatenated-batch layout
(h, g [A, nf]; pos, vel, box [A, 3]; N [M] atoms per molecule; r_cut [M]).
``Data.edges`` does NOT build an edge list on the host: it returns an
``Edges`` handle that carries positions, boxes, cut-offs and molecule
offsets, and the HIP kernels build the periodic neighbour pairs on the device
(inside the fused flow, per layer).  ``Edges.row / col / coord_diff`` are
materialised on demand through enflow_neighbour_pairs_f32 for callers that
want the explicit list; they hold the same multiset of (row, col) edges as the
reference (base.py:122-144), ordered by (row, col) instead of by periodic
image.
"""
import torch

from .. import _lib
from ..utils.helpers import apply_pbc, mol_ptr_from_counts


class Edges:
    """Device-side neighbour list handle (reference: base.py:9-19)."""

    def __init__(self, pos, box, r_cut, N, mol_ptr=None, max_mol_atoms=None):
        self.pos = pos
        self.box = box
        self.r_cut = r_cut
        self.N = N
        self._ptr = mol_ptr
        self._max_n = max_mol_atoms
        self._pairs = None

    # ---- metadata used by the kernels
    @property
    def mol_ptr(self):
        if self._ptr is None:
            self._ptr = mol_ptr_from_counts(self.N, device=self.pos.device)
        return self._ptr

    @property
    def max_mol_atoms(self):
        if self._max_n is None:
            N = torch.as_tensor(self.N)
            self._max_n = int(N.max()) if N.numel() else 0
        return self._max_n

    @property
    def num_mols(self):
        return int(self.mol_ptr.numel() - 1)

    # ---- explicit list (materialised on demand)
    def _materialise_large(self, L, dev, M, n):
        """Systems past the fused kernels' LDS image: per-row (label, mult)
        words from enflow_neighbour_pairs_large_f32, merged per (row, col)."""
        A = self.pos.shape[0]
        pos = self.pos.to(torch.float32).contiguous()
        box = self.box.to(torch.float32).contiguous()
        rc = torch.as_tensor(self.r_cut, device=dev).to(torch.float32).reshape(-1).contiguous()
        ptr = self.mol_ptr
        npairs = torch.empty(max(A, 1), dtype=torch.int32, device=dev)
        words = torch.empty((max(A, 1), n), dtype=torch.int32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        ws = _lib.large_workspace(M, A, n, 1, dev)
        _lib.check(L.enflow_neighbour_pairs_large_f32(M, A, n, _lib.ptr(ptr), _lib.ptr(rc), _lib.ptr(box),
                                                      _lib.ptr(pos), _lib.ptr(npairs), _lib.ptr(words),
                                                      _lib.ptr(err), _lib.ptr(ws), ws.numel(),
                                                      _lib.stream_ptr(dev)), "enflow_neighbour_pairs_large_f32")
        _lib.raise_on_err(err)
        cnt = npairs[:A].long()
        valid = torch.arange(n, device=dev)[None, :] < cnt[:, None]
        w = words[:A][valid].long() & 0xFFFFFFFF
        row = torch.arange(A, device=dev).repeat_interleave(cnt)
        mol = torch.searchsorted(ptr.long(), row, right=True) - 1
        off = ptr[:-1].long()[mol]
        col = ((w >> 5) & 0x3FFFFF) + off
        key, inv = torch.unique(row * max(A, 1) + col, return_inverse=True)
        mult = torch.zeros(key.numel(), dtype=torch.long, device=dev).index_add_(0, inv, w >> 27)
        row, col = key // max(A, 1), key % max(A, 1)
        mol = torch.searchsorted(ptr.long(), row, right=True) - 1
        return row, col, mult, mol

    def _materialise(self):
        if self._pairs is not None:
            return self._pairs
        L = _lib.lib()
        _lib.require_gpu(self.pos)
        dev = self.pos.device
        M = self.num_mols
        n = self.max_mol_atoms
        if _lib.is_large(n):
            self._pairs = self._materialise_large(L, dev, M, n)
            return self._pairs
        max_pairs = max(n * (n - 1), 1)
        pairs = torch.empty((M, max_pairs), dtype=torch.int32, device=dev)
        count = torch.empty(M, dtype=torch.int32, device=dev)
        err = torch.zeros(1, dtype=torch.int32, device=dev)
        pos = self.pos.to(torch.float32).contiguous()
        box = self.box.to(torch.float32).contiguous()
        rc = torch.as_tensor(self.r_cut, device=dev).to(torch.float32).reshape(-1).contiguous()
        ptr = self.mol_ptr
        _lib.check(L.enflow_neighbour_pairs_f32(M, pos.shape[0], n, _lib.ptr(ptr), _lib.ptr(rc),
                                                _lib.ptr(box), _lib.ptr(pos), max_pairs,
                                                _lib.ptr(pairs), _lib.ptr(count), _lib.ptr(err),
                                                _lib.stream_ptr(dev)), "enflow_neighbour_pairs_f32")
        _lib.raise_on_err(err)
        cnt = count.long()
        valid = torch.arange(max_pairs, device=dev)[None, :] < cnt[:, None]
        p = pairs[valid].long()
        mol = torch.arange(M, device=dev).repeat_interleave(cnt)
        off = ptr[:-1].long()[mol]
        row = (p & 0xFF) + off
        col = ((p >> 8) & 0xFF) + off
        mult = p >> 16
        self._pairs = (row, col, mult, mol)
        return self._pairs

    @property
    def row(self):
        row, _, mult, _ = self._materialise()
        return row.repeat_interleave(mult)

    @property
    def col(self):
        _, col, mult, _ = self._materialise()
        return col.repeat_interleave(mult)

    @property
    def edge_box(self):
        """Per-edge box = first-atom box of the edge's molecule (base.py:130,140)."""
        _, _, mult, mol = self._materialise()
        first = self.box[self.mol_ptr[:-1].long()]
        return first[mol].repeat_interleave(mult, dim=0)

    @property
    def coord_diff(self):
        """base.py:15-19, half-box minimum image included."""
        d = self.pos[self.row] - self.pos[self.col]
        return apply_pbc(d, self.edge_box * 0.5)


class Data:
    """Batch of molecules (reference: base.py:21-144)."""

    def __init__(self, z=None, h=None, g=None, pos=None, vel=None, N=None, r_cut=None, box=None,
                 label=None, device='cpu'):
        self.z = z
        self.h = h
        self.g = g
        self.pos = pos
        self.vel = vel
        self.N = N
        self.r_cut = r_cut
        self.box = box
        self.label = label
        self.device = device
        self._ptr = None
        self._max_n = None

    @classmethod
    def from_arrays(cls, batch, device='cuda', dtype=torch.float32):
        """Build from the dict layout of enflow_amd.data.synthetic (numpy)."""
        t = lambda k: torch.as_tensor(batch[k], dtype=dtype, device=device)  # noqa: E731
        import numpy as np
        N = torch.as_tensor(np.diff(batch["mol_ptr"]), dtype=torch.long)
        d = cls(h=t("h"), g=t("g"), pos=t("pos"), vel=t("vel"), N=N, r_cut=t("r_cut"),
                box=t("box"), device=device)
        return d

    def get_mol(self, i):
        if torch.as_tensor(self.N).ndim == 0:
            return self
        s = int(self.N[:i].sum())
        e = s + int(self.N[i])
        return Data(z=None if self.z is None else self.z[i], h=self.h[s:e], g=self.g[s:e],
                    pos=self.pos[s:e], vel=self.vel[s:e], N=self.N[i], r_cut=self.r_cut[i],
                    box=self.box[s:e], label=None if self.label is None else self.label[i],
                    device=self.device)

    @property
    def num_atoms(self):
        return int(torch.as_tensor(self.N).sum())

    @property
    def num_mols(self):
        N = torch.as_tensor(self.N)
        return 1 if N.ndim == 0 else len(N)

    def __iter__(self):
        self.i = 0
        return self

    def __next__(self):
        if self.i >= self.num_mols:
            raise StopIteration
        mol = self.get_mol(self.i)
        self.i += 1
        return mol

    def _replace(self, **kw):
        d = Data(z=self.z, h=self.h, g=self.g, pos=self.pos, vel=self.vel, N=self.N,
                 r_cut=self.r_cut, box=self.box, label=self.label, device=self.device)
        d._ptr, d._max_n = self._ptr, self._max_n
        for k, v in kw.items():
            setattr(d, k, v)
        return d

    def clone(self):
        return self._replace(h=self.h.clone(), g=self.g.clone(), pos=self.pos.clone(),
                             vel=self.vel.clone(), N=torch.as_tensor(self.N).clone(),
                             r_cut=torch.as_tensor(self.r_cut).clone(), box=self.box.clone())

    def to(self, device):
        d = self._replace(h=self.h.to(device), g=self.g.to(device), pos=self.pos.to(device),
                          vel=self.vel.to(device), N=torch.as_tensor(self.N),
                          r_cut=torch.as_tensor(self.r_cut).to(device), box=self.box.to(device))
        d.device = device
        d._ptr = None
        return d

    def pbc(self):
        self.pos = apply_pbc(self.pos, self.box)

    # ---- kernel metadata
    @property
    def mol_ptr(self):
        if self._ptr is None or self._ptr.device != self.pos.device:
            self._ptr = mol_ptr_from_counts(self.N, device=self.pos.device)
        return self._ptr

    @property
    def max_mol_atoms(self):
        if self._max_n is None:
            N = torch.as_tensor(self.N)
            self._max_n = int(N.max()) if N.numel() else 0
        return self._max_n

    @property
    def edges(self):
        return Edges(self.pos, self.box, self.r_cut, self.N, mol_ptr=self.mol_ptr,
                     max_mol_atoms=self.max_mol_atoms)


class DataLoader(torch.utils.data.DataLoader):
    """torch DataLoader with the reference's concatenating collater (base.py:146-174)."""

    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, **kwargs):
        super().__init__(dataset, batch_size, shuffle, collate_fn=self.collater, **kwargs)

    @staticmethod
    def collater(dataset):
        return Data(
            z=[d.z for d in dataset],
            h=torch.cat([d.h for d in dataset]),
            g=torch.cat([d.g for d in dataset]),
            pos=torch.cat([d.pos for d in dataset]),
            vel=torch.cat([d.vel for d in dataset]),
            N=torch.tensor([int(d.N) for d in dataset]),
            r_cut=torch.tensor([float(d.r_cut) for d in dataset]),
            box=torch.cat([d.box for d in dataset]),
            label=[d.label for d in dataset],
        )
