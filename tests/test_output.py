"""On-disk formats (pyrmt_amd/output.py): the reference's CSV layouts
byte for byte, and the snapshot round trip (HDF5 when h5py is present, .npz otherwise)."""
import csv
import io
import os

import numpy as np
import pytest


def test_centroid_csv_layout(tmp_path):
    from pyrmt_amd.output import write_centroid_csv
    traj = np.array([[0.001, 0.6, 0.5, 0.99, 1.01], [0.002, 0.6001, 0.5002, 0.98, 1.02]])
    p = tmp_path / "centroid.csv"
    write_centroid_csv(str(p), traj)
    # the reference's call (soft_disc_in_lid_driven.py:126-127) on the same rows
    buf = io.StringIO()
    np.savetxt(buf, traj, delimiter=",", header="t,cx,cy,minJ,maxJ", comments="")
    assert p.read_text() == buf.getvalue()
    back = np.loadtxt(str(p), delimiter=",", skiprows=1)
    np.testing.assert_array_equal(back, traj)


def test_energy_history_rows(tmp_path):
    from pyrmt_amd.output import append_energy_row, ENERGY_FIELDS
    d = str(tmp_path / "run")
    for step in (1, 100, 200):
        path = append_energy_row(d, step, 0.1 * step, 1e-3, 2.0, 3.0, 0.5, 0.25)
    rows = list(csv.reader(open(path)))
    assert rows[0] == ENERGY_FIELDS and len(rows) == 4
    assert rows[1][0] == "1" and float(rows[1][-1]) == 2.0 + 3.0 + 0.25
    # output.py:286: step 1 writes a header again even into an existing file
    append_energy_row(d, 1, 0.0, 1e-3, 1.0, 1.0, 0.0, 0.0)
    rows = list(csv.reader(open(path)))
    assert rows[4] == ENERGY_FIELDS


def test_snapshot_roundtrip(tmp_path):
    from pyrmt_amd.output import write_snapshot, read_snapshot
    rng = np.random.default_rng(0)
    ds = {"phi": rng.standard_normal((5, 5)), "a": rng.standard_normal((5, 5))}
    out = write_snapshot(str(tmp_path / "snap_t01.00.h5"), ds, {"t": 1.0001, "t_target": 1.0})
    got, attrs = read_snapshot(out)
    for k in ds:
        np.testing.assert_array_equal(got[k], ds[k])
    assert attrs["t"] == 1.0001 and attrs["t_target"] == 1.0


@pytest.mark.gpu
def test_snapshot_of_device_state(gpu, tmp_path):
    from pyrmt_amd.output import snapshot_sim, read_snapshot, trajectory, SNAPSHOT_FIELDS
    from pyrmt_amd.simulation import soft_disc_in_lid_driven
    sim = soft_disc_in_lid_driven(64)
    sim.step(3)
    got, attrs = read_snapshot(snapshot_sim(sim, str(tmp_path), 0.0))
    for name in SNAPSHOT_FIELDS:
        np.testing.assert_array_equal(got[name], sim.get(name))
    assert attrs["t"] == sim.diagnostics()["t"][-1]
    tr = trajectory(sim)
    assert tr.shape == (3, 5) and np.all(np.isfinite(tr))


def _osd_args(z):
    kw = {k[3:]: float(z[k]) for k in z.files if k.startswith("kw_")}
    return (float(z["dx"]), float(z["dy"]), z["phi"], z["solid"], z["X1"], z["X2"], z["a"],
            z["b"], z["p"]), (z["sxx"], z["sxy"], z["syy"], z["J"]), kw


def test_output_simulation_data_oracle_vs_reference_fixture(oracle):
    """The fixture (tests/golden/gen_golden.py gen_output: the reference's writer with a
    recording h5py) against the oracle's restatement: div_vel and the energies bit-exact."""
    from conftest import golden
    z = golden("output_sim")
    (dx, dy, phi, solid, X1, X2, a, b, p), (sxx, sxy, syy, J), kw = _osd_args(z)
    d, _ = oracle.divergence_2d_interior(a, b, dx, dy, pad=4)
    np.testing.assert_array_equal(d, z["ds_div_vel"])
    assert oracle.compute_kinetic_energy(a, b, kw["rho_f"], kw["rho_s"], phi, kw["w_t"], dx, dy) \
        == float(z["at_kinetic_energy"])
    assert oracle.compute_strain_energy(X1, X2, phi, kw["mu_s"], dx, dy, kappa=kw["kappa"]) \
        == float(z["at_strain_energy"])


@pytest.mark.gpu
def test_output_simulation_data_vs_reference(gpu, tmp_path, monkeypatch, capsys):
    """output.py:213-321 under its own name: the data_NNNNNN file's datasets (div_vel from
    the device, bit-exact) and attrs (energies at the A26 bars: KE / dissipation 1e-14
    relative -- device sin in the Heaviside --, SE bit-exact), the CSV rows and the log line
    against the reference's own output on the same inputs."""
    from conftest import golden
    from pyrmt_amd.output import output_simulation_data, read_snapshot
    z = golden("output_sim")
    args, tail, kw = _osd_args(z)
    monkeypatch.chdir(tmp_path)
    kws = dict(kw)
    ret = output_simulation_data(*args, 5, "case", 1, 2.5e-3, *tail, **kws)
    output_simulation_data(*args, 5, "case", 7, 2.5e-3, *tail, **kws)
    output_simulation_data(*args, 5, "case", 10, 2.5e-3, *tail, **kws)
    assert ret == float(z["ret"])
    out = capsys.readouterr().out
    assert out == str(z["log"])
    files = sorted(os.listdir(tmp_path / "outputs" / "case"))
    assert files[0] == "data_000001.h5" or files[0] == "data_000001.npz"
    assert len([f for f in files if f.startswith("data_")]) == 2
    ds, at = read_snapshot(str(tmp_path / "outputs" / "case" / files[0]))
    want_ds = {k[3:]: z[k] for k in z.files if k.startswith("ds_")}
    assert set(ds) == set(want_ds)
    for k, v in want_ds.items():
        np.testing.assert_array_equal(ds[k], v, err_msg=k)
    want_at = {k[3:]: float(z[k]) for k in z.files if k.startswith("at_")}
    assert set(at) == set(want_at)
    for k, v in want_at.items():
        np.testing.assert_allclose(float(at[k]), v, rtol=1e-14, err_msg=k)
    got_csv = list(csv.reader(open(tmp_path / "outputs" / "case" / "energy_history.csv")))
    want_csv = list(csv.reader(io.StringIO(str(z["csv"]))))
    assert got_csv[0] == want_csv[0] and len(got_csv) == len(want_csv)
    for g, w in zip(got_csv[1:], want_csv[1:]):
        np.testing.assert_allclose(np.array(g, float), np.array(w, float), rtol=1e-14)
