"""bench.py's evidence provenance: the rocprofv3 records
it quotes (profiles/traffic.json, profiles/valu.json, written by
tools/ingest_evidence.py) carry the build id of the library they profiled,
and bench.py marks a record of another build ``stale`` (its traffic is then
not quoted).  Host logic only."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_profile_records_are_matched_by_build_id(tmp_path, monkeypatch):
    sys.path.insert(0, REPO)
    import bench
    (tmp_path / 'profiles').mkdir()
    rec = {'bytes': 1.0e7, 'build_id': 'aaaa', 'source': 'profiles/rXX'}
    (tmp_path / 'profiles' / 'traffic.json').write_text(json.dumps({'K/fp64/4096': rec}))
    monkeypatch.setattr(bench, 'REPO', str(tmp_path))
    same = bench._profile_record('traffic.json', 'K/fp64/4096', 'aaaa')
    other = bench._profile_record('traffic.json', 'K/fp64/4096', 'bbbb')
    assert same['stale'] is False and same['bytes'] == 1.0e7
    assert other['stale'] is True
    assert bench._profile_record('traffic.json', 'missing', 'aaaa') is None
    assert bench._profile_record('valu.json', 'K/fp64/4096', 'aaaa') is None


def test_committed_records_name_their_build():
    """every committed record says which build it measured and where its
    evidence lies"""
    for name in ('traffic.json', 'valu.json'):
        db = json.load(open(os.path.join(REPO, 'profiles', name)))
        for key, rec in db.items():
            if rec.get('build_id') is None:      # round-3 records predate the stamping
                assert rec['source'].startswith('profiles/r03'), (name, key)
                continue
            assert len(rec['build_id']) == 16, (name, key)
            assert os.path.isdir(os.path.join(REPO, rec['source'])), (name, key, rec['source'])
