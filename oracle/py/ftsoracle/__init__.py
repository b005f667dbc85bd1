"""ftsoracle -- CPU restatement of the zkatdlog (nogh) crypto hot path.

TEST INFRASTRUCTURE ONLY.  Nothing under ``oracle/`` is part of the product:
only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import it, and only as the checker (or the timed CPU baseline), never
as the thing measured or shipped.

The reference (sudo-monkey/fabric-token-sdk, Go) cannot be built or run here:
no Go toolchain and the pinned modules ``github.com/IBM/mathlib
v0.0.0-20220112091634-0a7378db6912`` and ``github.com/consensys/gnark-crypto
v0.6.0`` are not on disk.  This package restates:

* ``bn254``   -- the BN254 arithmetic mathlib/gnark provide (Fp, Fp2/6/12 tower,
                 G1, G2, optimal-ate Miller loop, final exponentiation, the
                 gnark byte encodings) from the published algorithms;
* ``gojson``  -- the subset of Go ``encoding/json`` semantics the proof wire
                 format exercises (case-insensitive keys, null -> nil, base64
                 []byte, last-duplicate-wins);
* ``zkat``    -- the zkatdlog prover/verifier logic, following the reference
                 files cited function by function.

Parity status: accept/reject behaviour is pinned by the reference's own test
cases and curve known-answer facts; byte-level parity at
the mathlib boundary (GT byte order, final-exponent variant, JSON element
encoding) is **unpinned** -- the reference holds no golden vectors.
"""
