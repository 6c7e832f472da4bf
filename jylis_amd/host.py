"""Python handle over the C++ host mirror (include/jylis_host.h).

`Database` mirrors jylis/database.pony: `apply(*words)` answers one parsed
RESP command with RESP bytes, `flush()` returns the node's pending delta
batches as one blob (Database.flush_deltas, database.pony:42-48), and
`converge(blob)` folds a peer's blob in (Database.converge_deltas,
database.pony:50-51).  State lives on the GPU engine.
"""
import ctypes as C

from . import _lib


class Database:
    def __init__(self, device=0, identity=1):
        self.lib = _lib.load()
        h = C.c_void_p()
        rc = self.lib.jyh_db_create(device, identity & (2**64 - 1), C.byref(h))
        if rc != 0 or not h.value:
            raise RuntimeError(f"jyh_db_create failed ({rc}): no GPU / engine")
        self.h = h

    def close(self):
        if getattr(self, "h", None):
            self.lib.jyh_db_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def apply(self, *words):
        ws = [w.encode() if isinstance(w, str) else bytes(w) for w in words]
        argv = (C.c_char_p * len(ws))(*ws)
        lens = (C.c_uint64 * len(ws))(*[len(w) for w in ws])
        cap = 1 << 16
        while True:
            buf = C.create_string_buffer(cap)
            n = C.c_uint64()
            rc = self.lib.jyh_db_apply(self.h, len(ws), argv, lens, buf, cap, C.byref(n))
            if rc == -4 and n.value > cap:  # JY_ERANGE: grow the reply buffer
                cap = n.value
                continue
            if rc != 0:
                raise RuntimeError(self.lib.jyh_db_error(self.h).decode())
            return buf.raw[: n.value]

    def flush(self):
        p = C.c_void_p()
        n = C.c_uint64()
        self.lib.jyh_db_flush(self.h, C.byref(p), C.byref(n))
        out = C.string_at(p, n.value)
        self.lib.jyh_free(p)
        return out

    def converge(self, blob):
        rc = self.lib.jyh_db_converge(self.h, blob, len(blob))
        if rc != 0:
            raise RuntimeError(self.lib.jyh_db_error(self.h).decode())

    def shutdown(self):
        self.lib.jyh_db_shutdown(self.h)
