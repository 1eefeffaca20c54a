"""Per-kernel VGPR / spill / LDS metadata of two libjr.so builds (the code
objects' notes), printing the kernels whose numbers differ -- a register
budget that crosses an occupancy step (256 -> 257 VGPRs: 2 -> 1 waves per
SIMD) is what made the first counting stream-K hand-off 8 % slower.
python tools/kernel_meta.py <old libjr.so> <new libjr.so>"""
import subprocess, re, sys
def meta(so):
    tmp='/tmp/kmeta_'+str(abs(hash(so)))
    subprocess.run(['mkdir','-p',tmp])
    subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-objcopy','--dump-section','.hip_fatbin='+tmp+'/fat.bin',so,'/dev/null'],check=True)
    data=open(tmp+'/fat.bin','rb').read()
    magic=b'__CLANG_OFFLOAD_BUNDLE__'
    idx=[m.start() for m in re.finditer(re.escape(magic), data)]
    out={}
    for k,i in enumerate(idx):
        j=idx[k+1] if k+1<len(idx) else len(data)
        open(f'{tmp}/b{k}.bin','wb').write(data[i:j])
        r=subprocess.run(['/opt/rocm/lib/llvm/bin/clang-offload-bundler','--unbundle','--type=o',f'--input={tmp}/b{k}.bin','--targets=hipv4-amdgcn-amd-amdhsa--gfx950',f'--output={tmp}/c{k}.co'],capture_output=True)
        if r.returncode: continue
        notes=subprocess.run(['/opt/rocm/lib/llvm/bin/llvm-readelf','--notes',f'{tmp}/c{k}.co'],capture_output=True,text=True).stdout
        # parse kernel entries
        for blk in notes.split('  - .agpr_count')[1:]:
            name=re.search(r'\.name:\s+(\S+)',blk); v=re.search(r'\.vgpr_count:\s+(\d+)',blk); sp=re.search(r'\.vgpr_spill_count:\s+(\d+)',blk); a=re.search(r'^:\s+(\d+)',blk)
            lds=re.search(r'\.group_segment_fixed_size:\s+(\d+)',blk)
            if name and v: out[name.group(1)]=(int(v.group(1)), int(sp.group(1)) if sp else -1, int(lds.group(1)) if lds else -1)
    return out
a=meta(sys.argv[1]); b=meta(sys.argv[2])
import subprocess as sp
for n in sorted(set(a)&set(b)):
    if a[n]!=b[n] and 'k_conv' in n:
        dn=sp.run(['c++filt',n],capture_output=True,text=True).stdout.strip()
        print(a[n], '->', b[n], dn[:100])
