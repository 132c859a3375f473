# Records what Cython emits for the reference's n-step statement
# (dataset.pyx:1325: `n_step_return += reward * gamma ** i` with C float
# gamma / reward, C int i) — on a self-written three-line snippet, not on
# reference code.  Cython 0.29.21 (the reference's pin) is not installed; the
# installed Cython 3 reproduces 0.29's power semantics with the cpow=True
# directive, and its default (cpow=False) is shown for contrast.
set -e
T=$(mktemp -d)
cat > $T/probe.pyx <<'PYX'
cdef float step(float acc, float reward, float gamma, int i) nogil:
    acc += reward * gamma ** i
    return acc
PYX
{ echo "# cython: cpow=True"; cat $T/probe.pyx; } > $T/probe_legacy.pyx
python -m cython -3 $T/probe.pyx -o $T/probe.c >/dev/null
python -m cython -3 $T/probe_legacy.pyx -o $T/probe_legacy.c >/dev/null
echo "cython $(python -c 'import Cython; print(Cython.__version__)')"
echo "cpow=True (0.29 semantics):  $(grep '__pyx_v_acc = (' $T/probe_legacy.c | sed 's/^ *//')"
echo "cpow=False (Cython 3 default): $(grep '__pyx_v_acc = (' $T/probe.c | sed 's/^ *//')"
rm -rf $T
