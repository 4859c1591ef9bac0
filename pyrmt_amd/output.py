"""On-disk formats of the reference drivers, written from device state.

* ``centroid.csv`` -- benchmarks/soft_disc_in_lid_driven.py:125-127: the trajectory rows
  (t, cx, cy, minJ, maxJ) through ``np.savetxt(..., delimiter=",", header=..., comments="")``;
* ``energy_history.csv`` -- pyRMT/output.py:277-298: one row per output step appended with
  ``csv.DictWriter`` and the same field names (a header when the file is new, and again at
  step 1, as the reference does);
* snapshots -- soft_disc_in_lid_driven.py:110-118 (``snap_tXX.XX.h5``: phi, X1, X2, a, b, p,
  J, sigma_xx, sigma_xy, sigma_yy; attrs t, t_target) and ``output_simulation_data``
  (output.py:213-321, the reference's name and signature: ``data_NNNNNN.h5`` with phi, X1,
  X2, J, a, b, p, sigma_xx, sigma_yy, sigma_xy, div_vel and the attrs time, kinetic_energy,
  strain_energy, dissipation_rate, integrated_dissipation, total_energy; the energy row;
  the log line).  With h5py importable the same HDF5 layout is written; this image has no
  h5py, so the fallback is an ``.npz`` holding the same dataset names plus the attributes
  as ``attrs/<name>`` 0-d arrays (``read_snapshot`` reads either).

The arrays come from the device (``Simulation.get``); the energies and div_vel are computed
by librmt (compute_*_energy, divergence_2d_interior); the log line's maxima are formatting.
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


def output_simulation_data(dx, dy, phi, solid_mask, X1, X2, a, b, p, vis_output_freq,
                           directory_name, step, dt, sigma_sxx, sigma_sxy, sigma_syy, J,
                           mu_s=0.0, mu_f=0.0, rho_s=1.0, rho_f=1.0, w_t=None, eta_s=0.0,
                           kappa=0.0, time=0.0, integrated_dissipation=0.0):
    """output.py:213-321 (same signature, same files under outputs/<directory_name>):
    on output steps (step % vis_output_freq == 0 or step == 1) the energies, the log line,
    a row of energy_history.csv and data_{step:06d}.h5 (or .npz without h5py).  Returns
    integrated_dissipation (updated by the caller's loop, as in the reference)."""
    from .functions import (compute_kinetic_energy, compute_strain_energy,
                            compute_viscous_dissipation, divergence_2d_interior)
    if w_t is None:
        w_t = 2.0 * dx
    if not (step % vis_output_freq == 0 or step == 1):
        return integrated_dissipation
    host = lambda x: x.detach().cpu().numpy() if hasattr(x, "detach") else np.asarray(x)
    div_field, div_interior = divergence_2d_interior(a, b, dx, dy, pad=4)
    div_field, div_interior = host(div_field), host(div_interior)
    ke = compute_kinetic_energy(a, b, rho_f, rho_s, phi, w_t, dx, dy)
    se = compute_strain_energy(X1, X2, phi, mu_s, dx, dy, kappa=kappa)
    dissipation_rate = compute_viscous_dissipation(a, b, mu_f, phi, w_t, dx, dy, eta_s)
    total_energy = ke + se + integrated_dissipation
    ah, bh, Jh = host(a), host(b), host(J)
    sxx, sxy, syy = host(sigma_sxx), host(sigma_sxy), host(sigma_syy)
    vmag = np.sqrt(ah ** 2 + bh ** 2)
    print(f"[Step {step:05d}] t={time:.3f}, dt={dt:.2e}, "
          f"max|v|={np.max(vmag):.3f}, "
          f"KE={ke:.4e}, SE={se:.4e}, ε={dissipation_rate:.4e}, "
          f"E_tot={total_energy:.4e}, "
          f"min(J)={np.min(Jh):.3f}, "
          f"max|σ|={np.max(np.sqrt(sxx ** 2 + syy ** 2 + 2 * sxy ** 2)):.2f}, "
          f"max|div|={np.max(np.abs(div_interior)):.2e}")
    output_dir = os.path.join("outputs", directory_name)
    os.makedirs(output_dir, exist_ok=True)
    path = os.path.join(output_dir, "energy_history.csv")
    exists = os.path.isfile(path)
    with open(path, 'a', newline='') as f:
        w = csv.DictWriter(f, fieldnames=ENERGY_FIELDS)
        if not exists or step == 1:
            w.writeheader()
        w.writerow({'step': step, 'time': time, 'dt': dt, 'kinetic_energy': ke,
                    'strain_energy': se, 'dissipation_rate': dissipation_rate,
                    'integrated_dissipation': integrated_dissipation,
                    'total_energy': total_energy})
    ds = {"phi": host(phi), "X1": host(X1), "X2": host(X2), "J": Jh, "a": ah, "b": bh,
          "p": host(p), "sigma_xx": sxx, "sigma_yy": syy, "sigma_xy": sxy, "div_vel": div_field}
    write_snapshot(os.path.join(output_dir, f"data_{step:06d}.h5"), ds,
                   {'time': time, 'kinetic_energy': ke, 'strain_energy': se,
                    'dissipation_rate': dissipation_rate,
                    'integrated_dissipation': integrated_dissipation,
                    'total_energy': total_energy})
    return integrated_dissipation


def snapshot_sim(sim, out_dir, t_target):
    """The driver's field dump at a target time (soft_disc_in_lid_driven.py:110-118)."""
    os.makedirs(out_dir, exist_ok=True)
    d = sim.diagnostics()
    t = float(d["t"][-1]) if len(d["t"]) else 0.0
    ds = {name: sim.get(name) for name in SNAPSHOT_FIELDS}
    return write_snapshot(os.path.join(out_dir, f"snap_t{t_target:05.2f}.h5"), ds,
                          {"t": t, "t_target": t_target})
