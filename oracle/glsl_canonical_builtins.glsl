//@replace in vec2 FragCoord;	#define FragCoord gl_FragCoord

// ---- analysis prelude: the canonical builtins of include/ort_math.h (and the exact pixel centre) ----
const double ORT_LOG2_TAB[32] = double[32](1.3989071038251366LF, -0.4843001617159575LF, 1.3403141361256545LF, -0.4225711719642514LF, 1.2864321608040201LF, -0.3633753794563512LF, 1.2367149758454106LF, -0.3065130425006747LF, 1.1906976744186046LF, -0.2518071504105397LF, 1.147982062780269LF, -0.19910010007969525LF, 1.1082251082251082LF, -0.14825095858394247LF, 1.0711297071129706LF, -0.09913319201925132LF, 1.0364372469635628LF, -0.05163276841532236LF, 1.0LF, 0.0LF, 0.9481481481481482LF, 0.07681559705083084LF, 0.8951048951048951LF, 0.1598713367783894LF, 0.847682119205298LF, 0.2384047393250789LF, 0.8050314465408805LF, 0.3128829552843553LF, 0.7664670658682635LF, 0.38370429247405213LF, 0.7314285714285714LF, 0.4512111118323288LF);
const double ORT_EXP2_TAB[32] = double[32](1.0LF, 1.0218971486541166LF, 1.0442737824274138LF, 1.0671404006768237LF, 1.0905077326652577LF, 1.1143867425958924LF, 1.1387886347566916LF, 1.1637248587775775LF, 1.189207115002721LF, 1.215247359980469LF, 1.241857812073484LF, 1.2690509571917332LF, 1.2968395546510096LF, 1.3252366431597413LF, 1.3542555469368927LF, 1.383909881963832LF, 1.4142135623730951LF, 1.4451808069770467LF, 1.4768261459394993LF, 1.5091644275934228LF, 1.5422108254079407LF, 1.5759808451078865LF, 1.6104903319492543LF, 1.645755478153965LF, 1.681792830507429LF, 1.718619298122478LF, 1.7562521603732995LF, 1.7947090750031072LF, 1.8340080864093424LF, 1.8741676341103LF, 1.9152065613971474LF, 1.9571441241754002LF);
const double ORT_RNE = 6755399441055744.0LF;
float ort_nan() { return uintBitsToFloat(0x7fc00000u); }
float ort_inf() { return uintBitsToFloat(0x7f800000u); }
float ort_dot(vec3 a, vec3 b) { precise float r = (a.x * b.x + a.y * b.y) + a.z * b.z; return r; }
float ort_dot(vec2 a, vec2 b) { precise float r = a.x * b.x + a.y * b.y; return r; }
vec3 ort_normalize(vec3 v) { precise float s = 1.0 / sqrt(ort_dot(v, v)); precise vec3 r = v * s; return r; }
vec3 ort_cross(vec3 x, vec3 y) {
    precise vec3 r = vec3(x.y * y.z - y.y * x.z, x.z * y.x - y.z * x.x, x.x * y.y - y.x * x.y); return r; }
vec3 ort_reflect(vec3 i, vec3 n) { precise float k = 2.0 * ort_dot(n, i); precise vec3 r = i - k * n; return r; }
void ort_sincos(float xf, out float sn, out float cs) {
    if (isnan(xf) || isinf(xf)) { sn = ort_nan(); cs = ort_nan(); return; }
    precise double x = double(xf);
    precise double kd = (x * 0.6366197723675814LF + ORT_RNE) - ORT_RNE;
    precise double r = fma(-kd, 6.123233995736766e-17LF, fma(-kd, 1.5707963267948966LF, x));
    precise double z = r * r;
    precise double sp = fma(r * z, fma(z, fma(z, fma(z, 2.724920310940561e-06LF, -0.00019840081214087647LF),
                                         0.008333331864641476LF), -0.1666666666383007LF), r);
    precise double cp = fma(z, fma(z, fma(z, fma(z, 2.446300252898972e-05LF, -0.0013887583164707857LF),
                                   0.0416666505356106LF), -0.49999999968848047LF), 1.0LF);
    int q = int(kd) & 3;
    double sv = (q & 1) != 0 ? cp : sp, cv = (q & 1) != 0 ? sp : cp;
    sn = float((q & 2) != 0 ? -sv : sv);
    cs = float(((q + 1) & 2) != 0 ? -cv : cv);
}
float ort_sin(float x) { float s, c; ort_sincos(x, s, c); return s; }
float ort_cos(float x) { float s, c; ort_sincos(x, s, c); return c; }
float ort_tan(float x) { float s, c; ort_sincos(x, s, c); return float(double(s) / double(c)); }
double ort_log2_d(float xf) {
    uint ix = floatBitsToUint(xf);
    int ks = 0;
    if (ix < 0x00800000u) { float xs = xf * 8388608.0; ix = floatBitsToUint(xs); ks = -23; }
    uint tmp = ix - 0x3f330000u;
    int i = int((tmp >> 19) & 15u);
    uint iz = ix - (tmp & 0xff800000u);
    int k = (int(tmp) >> 23) + ks;
    float zf = uintBitsToFloat(iz);
    precise double r = fma(double(zf), ORT_LOG2_TAB[2 * i], -1.0LF);
    precise double p = r * fma(r, fma(r, fma(r, fma(r, 0.28881117497988373LF, -0.3609383389132996LF),
                                         0.4808982571575573LF), -0.7213474622454469LF), 1.4426950408933528LF);
    precise double res = (double(k) + ORT_LOG2_TAB[2 * i + 1]) + p;
    return res;
}
float ort_exp2_f(double t) {
    precise double kd = (t * 32.0LF + ORT_RNE) - ORT_RNE;
    precise double r = fma(kd, -0.03125LF, t);
    int ki = int(kd);
    precise double p = fma(r, fma(r, fma(r, 0.05550443425710469LF, 0.24022826844912404LF), 0.693147180550007LF), 1.0LF);
    uvec2 w = unpackDouble2x32(ORT_EXP2_TAB[ki & 31]);
    w.y += uint((ki >> 5) << 20);
    precise double res = packDouble2x32(w) * p;
    return float(res);
}
float ort_pow(float x, float y) {
    if (isnan(x) || isnan(y)) return ort_nan();
    if (x < 0.0) return ort_nan();
    if (y == 0.0) return 1.0;
    if (x == 0.0) return (y > 0.0) ? 0.0 : ort_inf();
    if (isinf(x)) return (y > 0.0) ? ort_inf() : 0.0;
    if (x == 1.0) return 1.0;
    precise double t = double(y) * ort_log2_d(x);
    if (t >= 128.0LF) return ort_inf();
    if (t <= -150.0LF) return 0.0;
    return ort_exp2_f(t);
}
vec3 ort_pow(vec3 x, vec3 y) { return vec3(ort_pow(x.x, y.x), ort_pow(x.y, y.y), ort_pow(x.z, y.z)); }
float ort_min(float x, float y) { return (y < x) ? y : x; }
float ort_max(float x, float y) { return (x < y) ? y : x; }
vec3 ort_min(vec3 x, vec3 y) { return vec3(ort_min(x.x, y.x), ort_min(x.y, y.y), ort_min(x.z, y.z)); }
vec3 ort_max(vec3 x, vec3 y) { return vec3(ort_max(x.x, y.x), ort_max(x.y, y.y), ort_max(x.z, y.z)); }
#define sin(x) ort_sin(x)
#define cos(x) ort_cos(x)
#define tan(x) ort_tan(x)
#define pow(x, y) ort_pow(x, y)
#define normalize(v) ort_normalize(v)
#define dot(a, b) ort_dot(a, b)
#define length(v) sqrt(ort_dot(v, v))
#define cross(a, b) ort_cross(a, b)
#define reflect(i, n) ort_reflect(i, n)
#define min(x, y) ort_min(x, y)
#define max(x, y) ort_max(x, y)
// ---- end of prelude ----
