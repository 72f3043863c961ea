function build_mpct_mex(repo)
% BUILD_MPCT_MEX  Compile the MEX gateway matlab/mpct_mex.c against libmpct.so.
%   build_mpct_mex(repo)  with repo = the root of this repository.  Build libmpct.so first
%   (python -c "import __graft_entry__ as g; g.build()"  ->  <repo>/model-predictive-control-
%   tuning_amd/csrc/libmpct.so; it links the HIP kernels of all five translation units).
if nargin < 1, repo = fileparts(fileparts(mfilename('fullpath'))); end
csrc = fullfile(repo, 'model-predictive-control-tuning_amd', 'csrc');
assert(isfile(fullfile(csrc, 'libmpct.so')), 'mpct:build', 'libmpct.so not built in %s', csrc);
mex('-R2018a', fullfile(repo, 'matlab', 'mpct_mex.c'), ['-I' fullfile(repo, 'include')], ...
    ['-L' csrc], '-lmpct', ['LDFLAGS=$LDFLAGS -Wl,-rpath,' csrc ' -Wl,-rpath,/opt/rocm/lib'], ...
    '-outdir', fullfile(repo, 'matlab'));
v = mpct_mex('version');
assert(v >= 7, 'mpct:abi', 'libmpct ABI %d, this MEX needs >= 7', v);
end
