// Links libgpu_nnue.so: GPU_NNUE_LIB_DIR, else the in-tree build (python -m fishnet_amd.build).
fn main() {
    let dir = std::env::var("GPU_NNUE_LIB_DIR").unwrap_or_else(|_| {
        let here = std::path::PathBuf::from(std::env::var("CARGO_MANIFEST_DIR").unwrap());
        here.join("../../fishnet_amd/lib").display().to_string()
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=gpu_nnue");
    println!("cargo:rerun-if-env-changed=GPU_NNUE_LIB_DIR");
    // the HIP runtime the library needs at run time (ROCm's default prefix)
    println!("cargo:rustc-link-search=native=/opt/rocm/lib");
}
