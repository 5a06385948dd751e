// Links the prebuilt HIP library the same way the app links its native Swift bridge
// (/root/reference/src-tauri/build.rs:114-239: cargo:rustc-link-search + cargo:rustc-link-lib).
// libspittle_hip.so is built by `make -C spittle_amd/csrc` (hipcc --offload-arch=gfx950).
fn main() {
    let dir = std::env::var("SPITTLE_HIP_LIB_DIR").unwrap_or_else(|_| {
        // default: the in-tree build next to this crate (rust/../spittle_amd)
        let here = std::env::var("CARGO_MANIFEST_DIR").expect("CARGO_MANIFEST_DIR");
        format!("{here}/../../spittle_amd")
    });
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=spittle_hip");
    // the app binary finds the library next to itself or in the build tree
    println!("cargo:rustc-link-arg=-Wl,-rpath,$ORIGIN");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=SPITTLE_HIP_LIB_DIR");
    println!("cargo:rerun-if-changed=../../include/spittle_hip.h");
}
