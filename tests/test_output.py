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
