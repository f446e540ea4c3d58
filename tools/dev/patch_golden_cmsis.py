p = '/root/repo/tests/golden/make_golden.py'
s = open(p).read()
old = '''def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit(f"{REF} missing: run `make -C oracle/ref` (needs /root/reference)")
'''
new = '''def make_cmsis():
    """CMSIS-DSP f32 golden vectors (uhsdr_ref dump=cmsis, oracle/ref/ref_cmsis.c): per case its
    parameters and every array, stored as tests/golden/cmsis_vectors.npz with keys
    '<case>.<field>' and a JSON manifest under 'manifest'."""
    with tempfile.TemporaryDirectory() as td:
        out = subprocess.run([REF, "dump=cmsis", f"out={td}"], check=True, capture_output=True, text=True).stdout
        man = json.loads(out)
        arrs = {}
        for case, d in man.items():
            for field, n in d["fields"].items():
                x = np.fromfile(os.path.join(td, f"{case}.{field}.f32"), dtype=np.float32)
                assert x.size == n, (case, field)
                arrs[f"{case}.{field}"] = x
    np.savez_compressed(os.path.join(HERE, "cmsis_vectors.npz"), manifest=json.dumps(man), **arrs)
    print(f"cmsis_vectors: {len(man)} cases")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=None)
    a = ap.parse_args()
    if not os.path.exists(REF):
        sys.exit(f"{REF} missing: run `make -C oracle/ref` (needs /root/reference)")
    if a.only == "cmsis":
        make_cmsis()
        return
    make_cmsis()
'''
assert old in s
s = s.replace(old, new)
open(p, 'w').write(s)
print("ok")
