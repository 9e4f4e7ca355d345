--[[
multigrid-poisson/hip.lua — drop-in GPU solver class for thenumbernine/lua-multigrid-poisson,
backed by libmgpoisson.so (include/mgpoisson.h) through LuaJIT FFI.

It accepts the constructor protocols of the reference:
  * cpu.lua table protocol (cpu.lua:173-216):
        local MG = require 'multigrid-poisson.hip'
        local mg = MG{size=n, maxiter=?, epsilon=?, errorCallback=function(iter, err) ... end, debug=?}
        mg:solve()            -- or mg:step() -> err
        mg:twoGrid(h, u, f)   -- u, f: lua-matrix-style 1-based tables u[i][j] (x = i), u updated in place
    mg.size is {n, n} (cpu.lua:178 matrix{size,size}); mg.smooth and mg.inPlaceIterativeSolver
    (MG.Jacobi | MG.GaussSeidel, cpu.lua:56-57) are writable: a change rebuilds the device context
    with psi and f kept.
  * cpu-raw.lua / gpu.lua positional protocol (cpu-raw.lua:142, 239; gpu.lua:26, 348):
        local mg = MG(size, real)    -- real = 'double' (default) or 'float'
        -- real = 'float' computes as cpu-raw.lua does (float images read into LuaJIT doubles: every
        -- expression in double, rounded at each store; arith = 'double'); MG{size=n, real='float',
        -- arith='real'} gives gpu.lua's float OpenCL arithmetic (gpu.lua:32), the table protocol's default
        mg:run()              -- two outer iterations, prints '#iter err'
        mg:twoGrid(h, uPtr, fPtr, L) -- raw real* host buffers of an L x L grid (cpu-raw.lua:186)
    Fields as cpu-raw.lua:148-171 names them, each an image-like {buffer=real*, width, height}
    downloaded on access: mg.psi, mg.f, mg.psiOld, mg.errorBuf, mg.tmpU, and per level size L
    mg.rs[L], mg.Rs[L], mg.vs[L], mg.Vs[L] (rs / vs computed on the device on request).
  * cpu-gpu.lua protocol (cpu-gpu.lua:55-72): MG(size, real, cpuDepth[, engine]) switches to the
    GPU's one-launch coarse engine at size 2^cpuDepth, or, given an engine with
    engine:twoGrid(h, uPtr, fPtr, L) (e.g. require'multigrid-poisson.cpu-raw'(2^cpuDepth)), hands
    that level's u and f to it and back, exactly as MultigridGPUSubset:twoGrid does.
  * Multi-GPU from this one Lua process (north_star: the V-cycle domain-decomposed across the
    node's GPUs): MG{size=n, dim=3, ngpu=8[, devices={...}], ...}.  The library builds the RCCL
    communicators (ncclCommInitAll) and runs every rank in its own host thread per call
    (mgp_group_*); fields are the global box.
mg:metrics() returns relErr, count, frobErr of the last outer iteration (gpu.lua:173-200);
mg:residualNorm() returns ||f - A psi||, ||f|| (device reduction).
Extra table fields select the build's configurations: dim (2|3), real, smoother ('jacobi'|'rbgs'|'gs_lex'),
cycle ('V'|'F'), prolong ('pc'|'linear'), coarse_init ('fresh'|'warm'), coarse_bc
('zero'|'consistent'), restriction ('average'|'full_weighting'), arith ('real'|'double'), device.
Defaults reproduce cpu.lua
(2D, double, Jacobi 7+7, V-cycle, injection, 2x2 average, fresh zero coarse guess, ghost value 0).
Errors from the library raise Lua errors (error()), as the reference's own failures do.

Not executable in this repository's CI (no Lua runtime in the image): tests/test_lua_binding.py
compiles the cdef below against include/mgpoisson.h, and ../mgpoisson/solver.py is the tested
Python twin of this file.
--]]
local ffi = require 'ffi'
local bit = require 'bit'

ffi.cdef[[
typedef struct mgp_ctx mgp_ctx;
typedef struct mgp_group mgp_group;
typedef struct mgp_opts {
    int32_t struct_size;
    int32_t dim;
    int64_t n[3];
    int32_t real_bytes;
    int32_t nu1, nu2;
    int32_t smoother;
    int32_t cycle;
    int32_t prolong;
    int32_t coarse_init;
    int32_t coarse_bc;
    int32_t coarse_sweeps;
    int32_t err_mode;
    int32_t device;
    int32_t rank, world;
    int32_t restriction;
    int64_t gather_cells;
    uint8_t comm_id[128];
    int32_t arith;
    int32_t api_version;
} mgp_opts;
int         mgp_version(void);
void        mgp_opts_default(mgp_opts* o);
int         mgp_create(mgp_ctx** out, const mgp_opts* o);
void        mgp_destroy(mgp_ctx* c);
const char* mgp_last_error(const mgp_ctx* c);
int         mgp_num_levels(const mgp_ctx* c);
int         mgp_level_info(const mgp_ctx* c, int level, int64_t info[8]);
int         mgp_init_point_charge(mgp_ctx* c);
int         mgp_set_field(mgp_ctx* c, int level, int which, const void* src, int64_t count, int mem);
int         mgp_get_field(const mgp_ctx* c, int level, int which, void* dst, int64_t count, int mem);
int         mgp_set_planes(mgp_ctx* c, int level, int which, int64_t z_begin, int64_t nz, const void* src, int mem);
int         mgp_get_planes(const mgp_ctx* c, int level, int which, int64_t z_begin, int64_t nz, void* dst, int mem);
int         mgp_cycle(mgp_ctx* c, double* err_out);
int         mgp_two_grid(mgp_ctx* c, double h, void* u, const void* f, int64_t L, int mem);
int         mgp_set_coarse_level(mgp_ctx* c, int64_t size);
typedef int (*mgp_coarse_fn)(void* user, double h, void* u, const void* f, int64_t size);
int         mgp_set_coarse_handoff(mgp_ctx* c, int64_t size, mgp_coarse_fn fn, void* user);
int         mgp_metrics(mgp_ctx* c, double* rel_err, int64_t* count, double* frob);
int         mgp_set_debug(mgp_ctx* c, int mode);
int         mgp_residual_norm(mgp_ctx* c, int level, double* rnorm, double* fnorm);
int         mgp_group_create(mgp_group** out, const mgp_opts* o, int ngpu, const int* devices);
mgp_ctx*    mgp_group_rank(mgp_group* g, int rank);
void        mgp_group_destroy(mgp_group* g);
const char* mgp_group_last_error(const mgp_group* g);
int         mgp_group_init_point_charge(mgp_group* g);
int         mgp_group_cycle(mgp_group* g, double* err_out);
int         mgp_group_cycles(mgp_group* g, int32_t k, double* errs);
int         mgp_group_set_field(mgp_group* g, int level, int which, const void* src, int64_t count, int mem);
int         mgp_group_get_field(mgp_group* g, int level, int which, void* dst, int64_t count, int mem);
int         mgp_group_residual_norm(mgp_group* g, int level, double* rnorm, double* fnorm);
]]

local lib = ffi.load(os.getenv('MGP_LIBRARY') or 'mgpoisson')

local CODES = {
	smoother = {jacobi = 0, rbgs = 1, gs_lex = 2},
	cycle = {V = 0, F = 1},
	prolong = {pc = 0, linear = 1},
	coarse_init = {fresh = 0, warm = 1},
	coarse_bc = {zero = 0, consistent = 1},
	restriction = {average = 0, full_weighting = 1},
	arith = {real = 0, double = 1},
}
-- include/mgpoisson.h MGP_FIELD_*; names of cpu-raw.lua:148-171
local FIELD = {psi = 0, f = 1, rs = 2, vs = 3, psiOld = 4, errorBuf = 5, tmpU = 6, Vs = 0, Rs = 1}

local function check(rc, ctx)
	if rc < 0 then error('libmgpoisson: ' .. ffi.string(lib.mgp_last_error(ctx)), 3) end
	return rc
end

local function checkGroup(rc, g)
	if rc < 0 then error('libmgpoisson: ' .. ffi.string(lib.mgp_group_last_error(g)), 3) end
	return rc
end

local MultigridHIP = {}
-- cpu.lua:56-57 inPlaceIterativeSolver values (functions there, markers here)
MultigridHIP.Jacobi = 'jacobi'
MultigridHIP.GaussSeidel = 'gs_lex'  -- cpu.lua:24-37's lexicographic in-place sweep, bit-identical (hyperplane order)
MultigridHIP.RedBlackGaussSeidel = 'rbgs'  -- the build's red/black form (the temporally blocked engines)

local LEVEL_FIELDS = {rs = true, Rs = true, vs = true, Vs = true}
local IMAGE_FIELDS = {psiOld = true, errorBuf = true, tmpU = true}

MultigridHIP.__index = function(self, k)
	if k == 'psi' or k == 'f' then
		if rawget(self, 'tableProtocol') then return self:getMatrix(FIELD[k]) end
		return self:getImage(FIELD[k], 0)
	end
	if k == 'psiBuffer' then return self:getBuffer(0) end
	if k == 'fBuffer' then return self:getBuffer(1) end
	if IMAGE_FIELDS[k] then return self:getImage(FIELD[k], 0) end
	if LEVEL_FIELDS[k] then
		local mg = self
		return setmetatable({}, {__index = function(_, L) return mg:getImage(FIELD[k], mg:levelOf(L)) end})
	end
	if k == 'inPlaceIterativeSolver' then
		return rawget(self, 'pendingSmoother') or rawget(self, 'build').smoother
	end
	-- the value last assigned, as a plain field of cpu.lua's object would read back
	if k == 'smooth' then return rawget(self, 'pendingSmooth') or rawget(self, 'build').smooth end
	return rawget(MultigridHIP, k)
end

MultigridHIP.__newindex = function(self, k, v)
	if k == 'smooth' then
		rawset(self, 'pendingSmooth', v)
	elseif k == 'inPlaceIterativeSolver' then
		local name = (v == MultigridHIP.GaussSeidel or v == 'GaussSeidel') and 'gs_lex' or
			((v == MultigridHIP.RedBlackGaussSeidel or v == 'RedBlackGaussSeidel') and 'rbgs' or
			((v == MultigridHIP.Jacobi or v == 'Jacobi') and 'jacobi' or
			error('inPlaceIterativeSolver: Jacobi | GaussSeidel | RedBlackGaussSeidel')))
		rawset(self, 'pendingSmoother', name)
	else
		rawset(self, k, v)
	end
end

-- class defaults (cpu.lua:18-22, cpu-raw.lua:121-124)
MultigridHIP.debug = false
-- cpu-raw.lua:121 / gpu.lua:21: check every phase's output for non-finite cells ("found a nan", cpu-raw.lua:135-139)
MultigridHIP.debugging = false
MultigridHIP.smooth = 7
MultigridHIP.epsilon = 1e-10
MultigridHIP.accuracy = 1e-10
MultigridHIP.maxiter = 1000

setmetatable(MultigridHIP, {
	__call = function(cls, ...)
		local self = setmetatable({}, cls)
		self:init(...)
		return self
	end,
})

function MultigridHIP:makeOpts()
	local b = rawget(self, 'build')
	local n, dim = rawget(self, 'n'), rawget(self, 'dim')
	local o = ffi.new('mgp_opts')
	lib.mgp_opts_default(o)
	o.dim = dim
	o.n[0], o.n[1], o.n[2] = n, n, (dim == 3 and n or 1)
	o.real_bytes = (b.real == 'float') and 4 or 8
	o.nu1, o.nu2 = b.smooth, b.smooth
	for field, map in pairs(CODES) do
		if b[field] ~= nil then o[field] = assert(map[b[field]], 'unknown ' .. field) end
	end
	if b.device then o.device = b.device end
	return o
end

function MultigridHIP:createContext()
	local o = self:makeOpts()
	local ngpu = rawget(self, 'ngpu')
	if ngpu and ngpu > 1 then
		local devs = rawget(self, 'devices')
		local darr = devs and ffi.new('int[?]', ngpu, devs) or nil
		local pp = ffi.new('mgp_group*[1]')
		checkGroup(lib.mgp_group_create(pp, o, ngpu, darr), nil)
		rawset(self, 'group', ffi.gc(pp[0], lib.mgp_group_destroy))
	else
		local pp = ffi.new('mgp_ctx*[1]')
		check(lib.mgp_create(pp, o), nil)
		rawset(self, 'ctx', ffi.gc(pp[0], lib.mgp_destroy))
		self:applyCoarse()
	end
end

-- cpu-gpu.lua:55-72 cpuDepth: the GPU's one-launch coarse engine from size 2^cpuDepth, or the hand-off of
-- that level to engine:twoGrid (re-applied whenever the context is rebuilt)
function MultigridHIP:applyCoarse()
	local cpuDepth, engine = rawget(self, 'cpuDepth'), rawget(self, 'engine')
	if not cpuDepth then return end
	local L = bit.lshift(1, cpuDepth)
	if engine then
		-- cpu-gpu.lua:17-52: the callback runs engine:twoGrid on the level's host copies
		local cb = rawget(self, 'handoff')
		if not cb then
			local pt = rawget(self, 'ptype')
			cb = ffi.cast('mgp_coarse_fn', function(user, h, u, f, size)
				local ok = pcall(engine.twoGrid, engine, h, ffi.cast(pt, u), ffi.cast(pt, f), tonumber(size))
				return ok and 0 or 1
			end)
			rawset(self, 'handoff', cb)  -- keep the callback alive
		end
		check(lib.mgp_set_coarse_handoff(self.ctx, L, cb, nil), self.ctx)
	else
		lib.mgp_set_coarse_level(self.ctx, L)  -- keeps the default switch when it does not fit
	end
end

function MultigridHIP:init(a, real, cpuDepth, engine)
	local args
	if type(a) == 'table' then
		args = a
		-- like cpu.lua:174-177: nil fields fall back to the class defaults
		rawset(self, 'tableProtocol', true)
		rawset(self, 'maxiter', args.maxiter)
		rawset(self, 'epsilon', args.epsilon)
		rawset(self, 'errorCallback', args.errorCallback)
		if args.debug ~= nil then rawset(self, 'debug', args.debug) end
	else
		-- cpu-raw.lua positional protocol: persistent coarse buffers (cpu-raw.lua:221) and, for
		-- real = 'float', its LuaJIT-double arithmetic over float images (cpu-raw.lua:142-153)
		args = {size = a, real = real, coarse_init = 'warm', arith = 'double'}
		rawset(self, 'cpuDepth', cpuDepth)
		rawset(self, 'engine', engine)
	end
	local n = assert(tonumber(args.size), 'size is required')
	local dim = args.dim or 2
	rawset(self, 'real', args.real or 'double')
	rawset(self, 'dim', dim)
	rawset(self, 'n', n)
	-- cpu.lua:178 self.size = matrix{size, size}; cpu-raw.lua:146 self.size = size
	rawset(self, 'size', rawget(self, 'tableProtocol') and {n, n} or n)
	rawset(self, 'ngpu', args.ngpu)
	rawset(self, 'devices', args.devices)
	local smoother = args.smoother
	if args.inPlaceIterativeSolver then
		local v = args.inPlaceIterativeSolver
		smoother = (v == MultigridHIP.GaussSeidel) and 'gs_lex' or
			((v == MultigridHIP.RedBlackGaussSeidel) and 'rbgs' or 'jacobi')
	end
	rawset(self, 'build', {real = rawget(self, 'real'), smooth = args.smooth or MultigridHIP.smooth,
		smoother = smoother or 'jacobi', cycle = args.cycle, prolong = args.prolong,
		coarse_init = args.coarse_init, coarse_bc = args.coarse_bc, restriction = args.restriction,
		arith = args.arith, device = args.device})
	local cells = n * n * (dim == 3 and n or 1)
	rawset(self, 'count', cells)
	rawset(self, 'ctype', (rawget(self, 'real') == 'float') and 'float[?]' or 'double[?]')
	rawset(self, 'ptype', (rawget(self, 'real') == 'float') and 'float*' or 'double*')
	self:createContext()
	self:initPointCharge()
end

function MultigridHIP:initPointCharge()
	local g = rawget(self, 'group')
	if g then checkGroup(lib.mgp_group_init_point_charge(g), g)
	else check(lib.mgp_init_point_charge(self.ctx), self.ctx) end  -- cpu.lua:180-193
end

-- a changed smooth / inPlaceIterativeSolver takes effect here (the reference reads them inside
-- every twoGrid call, cpu.lua:96, 161): the context is rebuilt around the current psi and f
function MultigridHIP:applyKnobs()
	local ns, nm = rawget(self, 'pendingSmooth'), rawget(self, 'pendingSmoother')
	if ns == nil and nm == nil then return end
	local psi, f = self:getBuffer(0), self:getBuffer(1)
	local b = rawget(self, 'build')
	if ns ~= nil then b.smooth = ns end
	if nm ~= nil then b.smoother = nm end
	rawset(self, 'pendingSmooth', nil)
	rawset(self, 'pendingSmoother', nil)
	rawset(self, 'ctx', nil)
	rawset(self, 'group', nil)
	collectgarbage()
	self:createContext()
	self:setBuffer(0, psi)
	self:setBuffer(1, f)
end

-- the context that answers level queries: the solver's own, or rank 0's of a multi-GPU group
function MultigridHIP:infoCtx()
	local g = rawget(self, 'group')
	if g then return lib.mgp_group_rank(g, 0) end
	return self.ctx
end

function MultigridHIP:levelOf(size)
	local info = ffi.new('int64_t[8]')
	local ctx = self:infoCtx()
	local n = check(lib.mgp_num_levels(ctx), ctx)
	for l = 0, n - 1 do
		check(lib.mgp_level_info(ctx, l, info), ctx)
		if tonumber(info[0]) == size then return l end
	end
	error('no level of size ' .. tostring(size))
end

function MultigridHIP:metrics()
	if rawget(self, 'group') then error('metrics: single-GPU solvers only (ngpu > 1 runs mgp_group_*)', 2) end
	local rel, n, frob = ffi.new('double[1]'), ffi.new('int64_t[1]'), ffi.new('double[1]')
	check(lib.mgp_metrics(self.ctx, rel, n, frob), self.ctx)
	return rel[0], tonumber(n[0]), frob[0]
end

function MultigridHIP:residualNorm(level)
	local r, f = ffi.new('double[1]'), ffi.new('double[1]')
	local g = rawget(self, 'group')
	if g then checkGroup(lib.mgp_group_residual_norm(g, level or 0, r, f), g)
	else check(lib.mgp_residual_norm(self.ctx, level or 0, r, f), self.ctx) end
	return r[0], f[0]
end

function MultigridHIP:getBuffer(which, level)
	level = level or 0
	local count = self.count
	if level ~= 0 then
		-- a group's fields are the global box: nz_global (info[2]); one context's are its planes (info[3])
		local info = ffi.new('int64_t[8]')
		local ctx = self:infoCtx()
		check(lib.mgp_level_info(ctx, level, info), ctx)
		count = tonumber(info[0] * info[1] * (rawget(self, 'group') and info[2] or info[3]))
	end
	local buf = ffi.new(self.ctype, count)
	local g = rawget(self, 'group')
	if g then checkGroup(lib.mgp_group_get_field(g, level, which, buf, count, 0), g)
	else check(lib.mgp_get_field(self.ctx, level, which, buf, count, 0), self.ctx) end
	return buf, count
end

function MultigridHIP:setBuffer(which, buf)
	local g = rawget(self, 'group')
	if g then checkGroup(lib.mgp_group_set_field(g, 0, which, buf, self.count, 0), g)
	else check(lib.mgp_set_field(self.ctx, 0, which, buf, self.count, 0), self.ctx) end
end

-- image-like view (cpu-raw.lua's image(w,h,1,real) with .buffer), a host copy
function MultigridHIP:getImage(which, level)
	local buf, count = self:getBuffer(which, level)
	local w = math.floor(math.sqrt(count) + 0.5)
	if self.dim == 3 then w = math.floor(count ^ (1 / 3) + 0.5) end
	return {buffer = buf, width = w, height = w, count = count}
end

-- 1-based nested table m[i][j] with i = x (cpu.lua's matrix indexing), 2D only
function MultigridHIP:getMatrix(which)
	local buf = self:getBuffer(which)
	local n = self.n
	if self.dim ~= 2 then return buf end
	local m = {}
	for i = 1, n do
		local row = {}
		for j = 1, n do row[j] = tonumber(buf[(i - 1) + n * (j - 1)]) end
		m[i] = row
	end
	return m
end

-- cpu.lua:196-206
function MultigridHIP:step()
	self:applyKnobs()
	local err = ffi.new('double[1]')
	local g = rawget(self, 'group')
	if g then checkGroup(lib.mgp_group_cycle(g, err), g)
	else check(lib.mgp_cycle(self.ctx, err), self.ctx) end
	if self.debug then print('err', err[0]) end
	return err[0]
end

local function finite(x) return x == x and x ~= math.huge and x ~= -math.huge end

-- cpu.lua:208-216, break rules included
function MultigridHIP:solve()
	if self.debug then print('#iter', 'err') end
	for iter = 1, self.maxiter do
		local err = self:step()
		if self.errorCallback and self.errorCallback(iter, err) then break end
		if err < self.epsilon or not finite(err) then break end
	end
end

-- cpu-raw.lua:239-258 / gpu.lua:348-373: two outer iterations
function MultigridHIP:run()
	if not rawget(self, 'group') then check(lib.mgp_set_debug(self.ctx, self.debugging and 1 or 0), self.ctx) end
	print('#iter', 'err')
	for iter = 1, 2 do
		local err = self:step()
		print(iter, err)
		if err < self.accuracy or not finite(err) then break end  -- gpu.lua:371 math.isfinite
	end
end

-- cpu-raw.lua:186 twoGrid(h, u, f, L) on raw host real* buffers (u updated in place), or
-- cpu.lua:70 twoGrid(h, u, f) on lua-matrix-style tables u[i][j] (x = i; u updated in place)
function MultigridHIP:twoGrid(h, u, f, L)
	self:applyKnobs()
	if type(u) == 'table' then
		local n = #u
		local ub, fb = ffi.new(self.ctype, n * n), ffi.new(self.ctype, n * n)
		for i = 1, n do
			for j = 1, n do
				ub[(i - 1) + n * (j - 1)] = u[i][j]
				fb[(i - 1) + n * (j - 1)] = f[i][j]
			end
		end
		check(lib.mgp_two_grid(self.ctx, h, ub, fb, n, 0), self.ctx)
		for i = 1, n do
			for j = 1, n do u[i][j] = tonumber(ub[(i - 1) + n * (j - 1)]) end
		end
		return u
	end
	check(lib.mgp_two_grid(self.ctx, h, u, f, L, 0), self.ctx)
end

return MultigridHIP
