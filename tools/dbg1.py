"""One-document SV + diff through the C ABI, HIP errors named (debugging aid)."""
import os
import sys

sys.path[:0] = ['y-crdt_amd', 'oracle', 'tests']
os.environ['YMERGE_VERBOSE'] = '1'
import ymerge  # noqa: E402

u = bytes.fromhex('0102050004010174036162638405020278770000')
try:
    print(ymerge.encode_state_vector_from_update_v1(u).hex(), flush=True)
    print(ymerge.diff_updates_v1(u, bytes.fromhex('00')).hex(), flush=True)
except Exception as e:  # noqa: BLE001
    print('err', e, flush=True)
    sys.exit(1)
