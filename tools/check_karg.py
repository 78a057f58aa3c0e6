"""Build-time guard of the kernarg-segment reads (KP() / CamRef, rtw_render.hip).

KP(field) and CamRef read KParams through __builtin_amdgcn_kernarg_segment_ptr(). That
pointer is the kernel's own argument block only inside the kernel's body: a helper the
compiler outlines gets some other value (round 5's noinline A/B build read garbage and
faulted with hipErrorIllegalAddress). karg_base() therefore tags every expansion with an
assembler comment carrying sizeof(KParams) ("; rtw-karg kparams=N"), and this checker
reads the device listing (`make asm`, build/rtw_render.s) and fails unless, for EVERY
function whose body holds the tag:
  1. the function is a kernel (it has an .amdhsa_kernel descriptor), not a callee;
  2. its body makes no call (s_swappc_b64 / s_setpc_b64 / s_call_b64);
  3. its argument block is exactly one by-value argument of N bytes at offset 0 (a lone
     KParams, so the offsets KP() adds are the struct's).
It also fails if the listing holds any non-kernel function at all: everything in the
render file is meant to be inlined, and a callee there is how rule 1 gets broken next.

Usage: python tools/check_karg.py build/rtw_render.s [--expect-fail]
Prints one line per tagged kernel (name, private segment size) and exits 1 on a
violation (0 with --expect-fail only if a violation was found: the self-test of
`make karg-selftest`, which builds a deliberately noinline helper).
"""
import re
import sys

TAG = re.compile(r';\s*rtw-karg kparams=(0x[0-9a-fA-F]+|\d+)')
CALL = re.compile(r'^\s*(s_swappc_b64|s_setpc_b64|s_call_b64)\b')


def parse(path):
    lines = open(path).read().split('\n')
    funcs = {}   # name -> (start, end) line range of the body
    for i, l in enumerate(lines):
        m = re.match(r'^\s*\.type\s+([\w.$]+),@function', l)
        if not m:
            continue
        name = m.group(1)
        st = next((j for j in range(i, len(lines)) if lines[j].startswith(name + ':')), None)
        if st is None:
            continue
        en = next((j for j in range(st, len(lines)) if lines[j].strip().startswith('.Lfunc_end')), len(lines))
        funcs[name] = (st, en)
    kernels = set(re.findall(r'^\s*\.amdhsa_kernel\s+([\w.$]+)', '\n'.join(lines), re.M))
    # metadata: per kernel its .args list and private segment size
    meta = {}
    text = '\n'.join(lines)
    mb = re.search(r'\.amdgpu_metadata(.*?)\.end_amdgpu_metadata', text, re.S)
    if mb:
        for entry in re.split(r'\n  - ', mb.group(1)):
            nm = re.search(r'\.name:\s+(\S+)', entry)
            if not nm:
                continue
            args_blk = re.search(r'\.args:\s*\n((?:\s{6,}.*\n?)*)', entry)
            args = []
            if args_blk:
                for a in re.split(r'\n\s*- ', '\n' + args_blk.group(1)):
                    off = re.search(r'\.offset:\s+(\d+)', a)
                    size = re.search(r'\.size:\s+(\d+)', a)
                    kind = re.search(r'\.value_kind:\s+(\S+)', a)
                    if off and size and kind:
                        args.append((int(off.group(1)), int(size.group(1)), kind.group(1)))
            priv = re.search(r'\.private_segment_fixed_size:\s+(\d+)', entry)
            meta[nm.group(1)] = (args, int(priv.group(1)) if priv else None)
    return lines, funcs, kernels, meta


def check(path):
    lines, funcs, kernels, meta = parse(path)
    errors, report = [], []
    for name, (st, en) in sorted(funcs.items(), key=lambda kv: kv[1][0]):
        body = lines[st:en]
        tags = {int(m.group(1), 0) for l in body for m in [TAG.search(l)] if m}
        calls = [l.strip() for l in body if CALL.match(l)]
        if name not in kernels:
            errors.append(f'{name}: a non-kernel function in the render file'
                          + (' that reads the kernarg segment (KP/CamRef)' if tags else ''))
            continue
        if not tags:
            continue
        if len(tags) != 1:
            errors.append(f'{name}: inconsistent KParams sizes {sorted(tags)}')
        if calls:
            errors.append(f'{name}: reads the kernarg segment and makes calls ({calls[0]})')
        args, priv = meta.get(name, (None, None))
        # the compiler's hidden arguments (grid sizes, dynamic LDS size) follow the block
        args = [a for a in (args or []) if not a[2].startswith('hidden_')]
        want = [(0, next(iter(tags)), 'by_value')]
        if args != want:
            errors.append(f'{name}: reads KParams through the kernarg segment but its arguments are {args}, '
                          f'not one by-value KParams {want}')
        report.append(f'  {name}: KParams {next(iter(tags))} B, private segment {priv} B')
    if not report and not errors:
        errors.append('no function carries the rtw-karg tag: the listing is not the render file, or the tag '
                      'was lost')
    return errors, report


def main(argv):
    path = argv[1]
    expect_fail = '--expect-fail' in argv
    errors, report = check(path)
    if expect_fail:
        if errors:
            print('karg guard self-test: violation detected as required:\n  ' + '\n  '.join(errors))
            return 0
        print('karg guard self-test FAILED: the deliberately outlined helper was not detected')
        return 1
    if errors:
        print('karg guard FAILED (rtw_render.hip KP()/CamRef read the kernarg segment outside a '
              'lone-KParams kernel body):\n  ' + '\n  '.join(errors))
        return 1
    print(f'karg guard ok: {len(report)} kernels read KParams in their own bodies, no calls')
    print('\n'.join(report))
    return 0


if __name__ == '__main__':
    sys.exit(main(sys.argv))
