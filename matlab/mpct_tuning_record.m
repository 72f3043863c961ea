function Tuning_Parameters = mpct_tuning_record(matfile, mpcobj)
% MPCT_TUNING_RECORD  Complete a Tuning_Parameters .mat written by the engine's Python tuner
% (mpct.tuning.save_tuning_parameters: N, Nu, delta, lambda, scale.{L,R,Ru,Rv}, date as a datenum)
% into the record MPCTuning.m:374-381 saves: the mpc object with the tuned horizons and weights
% (MATLAB-only, so the Python side cannot write it) and date as a datetime.  The drivers'
% tuning = false path (Shell3x3.m:169-185) then loads it unchanged.
S = load(matfile, 'Tuning_Parameters');
T = S.Tuning_Parameters;
mpcobj.PredictionHorizon = max(T.N);
mpcobj.ControlHorizon = max(T.Nu);
mpcobj.Weights.OV = T.delta;
mpcobj.Weights.MVRate = T.lambda;
T.mpcobj = mpcobj;
if isnumeric(T.date), T.date = datetime(T.date, 'ConvertFrom', 'datenum'); end
Tuning_Parameters = T;
save(matfile, 'Tuning_Parameters');
end
