"""Content hash of the native sources, baked into the built extension to detect stale builds."""
import hashlib
import os


def source_hash(*src_dirs: str) -> str:
    h = hashlib.sha256()
    for src_dir in src_dirs:
        for name in sorted(os.listdir(src_dir)):
            if name.endswith((".hip", ".cpp", ".h")):
                h.update(name.encode())
                with open(os.path.join(src_dir, name), "rb") as f:
                    h.update(f.read())
    return h.hexdigest()[:16]
