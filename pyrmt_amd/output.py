"""On-disk formats of the reference drivers, written from device state.

* ``centroid.csv`` -- benchmarks/soft_disc_in_lid_driven.py:125-127: the trajectory rows
  (t, cx, cy, minJ, maxJ) through ``np.savetxt(..., delimiter=",", header=..., comments="")``;
* ``energy_history.csv`` -- pyRMT/output.py:277-298: one row per output step appended with
  ``csv.DictWriter`` and the same field names (a header when the file is new, and again at
  step 1, as the reference does);
* snapshots -- soft_disc_in_lid_driven.py:110-118 (``snap_tXX.XX.h5``: phi, X1, X2, a, b, p,
  J, sigma_xx, sigma_xy, sigma_yy; attrs t, t_target) and output.py:300-320
  (``data_NNNNNN.h5``).  With h5py importable the same HDF5 layout is written; this image
  has no h5py, so the fallback is an ``.npz`` holding the same dataset names plus the
  attributes as ``attrs/<name>`` 0-d arrays (``read_snapshot`` reads either).

The arrays come from the device (``Simulation.get``); nothing here computes physics.
"""
import csv
import os

import numpy as np

ENERGY_FIELDS = ['step', 'time', 'dt', 'kinetic_energy', 'strain_energy', 'dissipation_rate',
                 'integrated_dissipation', 'total_energy']
SNAPSHOT_FIELDS = ("phi", "X1", "X2", "a", "b", "p", "J", "sigma_xx", "sigma_xy", "sigma_yy")


def _h5py():
    try:
        import h5py
        return h5py
    except ImportError:
        return None


def write_centroid_csv(path, traj):
    """soft_disc_in_lid_driven.py:126-127."""
    np.savetxt(path, np.asarray(traj), delimiter=",", header="t,cx,cy,minJ,maxJ", comments="")


def trajectory(sim):
    """(t, cx, cy, minJ, maxJ) rows of a Simulation's per-step diagnostics (:107)."""
    d = sim.diagnostics()
    return np.stack([d["t"], d["cx"], d["cy"], d["minJ"], d["maxJ"]], axis=1)


def append_energy_row(output_dir, step, time, dt, kinetic_energy, strain_energy,
                      dissipation_rate, integrated_dissipation):
    """output.py:277-298 (total = KE + SE + integrated dissipation, :260)."""
    os.makedirs(output_dir, exist_ok=True)
    path = os.path.join(output_dir, "energy_history.csv")
    exists = os.path.isfile(path)
    with open(path, 'a', newline='') as f:
        w = csv.DictWriter(f, fieldnames=ENERGY_FIELDS)
        if not exists or step == 1:
            w.writeheader()
        w.writerow({'step': step, 'time': time, 'dt': dt, 'kinetic_energy': kinetic_energy,
                    'strain_energy': strain_energy, 'dissipation_rate': dissipation_rate,
                    'integrated_dissipation': integrated_dissipation,
                    'total_energy': kinetic_energy + strain_energy + integrated_dissipation})
    return path


def write_snapshot(path, datasets, attrs):
    """HDF5 (h5py) with `datasets` and `attrs`, else <path stem>.npz; returns the path
    written."""
    h5py = _h5py()
    if h5py is not None:
        with h5py.File(path, "w") as f:
            for k, v in datasets.items():
                f.create_dataset(k, data=np.asarray(v))
            for k, v in attrs.items():
                f.attrs[k] = v
        return path
    out = os.path.splitext(path)[0] + ".npz"
    arrs = {k: np.asarray(v) for k, v in datasets.items()}
    arrs.update({f"attrs/{k}": np.asarray(v) for k, v in attrs.items()})
    np.savez(out, **arrs)
    return out


def read_snapshot(path):
    """(datasets, attrs) from a file written by write_snapshot (either format)."""
    if path.endswith(".npz"):
        with np.load(path, allow_pickle=False) as z:
            ds = {k: z[k] for k in z.files if not k.startswith("attrs/")}
            at = {k[6:]: z[k][()] for k in z.files if k.startswith("attrs/")}
        return ds, at
    h5py = _h5py()
    with h5py.File(path, "r") as f:
        return {k: f[k][()] for k in f.keys()}, dict(f.attrs)


def snapshot_sim(sim, out_dir, t_target):
    """The driver's field dump at a target time (soft_disc_in_lid_driven.py:110-118)."""
    os.makedirs(out_dir, exist_ok=True)
    d = sim.diagnostics()
    t = float(d["t"][-1]) if len(d["t"]) else 0.0
    ds = {name: sim.get(name) for name in SNAPSHOT_FIELDS}
    return write_snapshot(os.path.join(out_dir, f"snap_t{t_target:05.2f}.h5"), ds,
                          {"t": t, "t_target": t_target})
